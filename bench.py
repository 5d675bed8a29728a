"""Benchmark: training-step spectrogram-frames/s (BASELINE.json metric), MI355X.

Workload (BASELINE.json configs[2] / SURVEY 8(d) config 3): one PerformanceNet training
step per GPU on a batch of 32 synthetic 4 s @ 16 kHz piano clips (L = 64,256 samples,
T = 252 frames): on-the-fly STFT log-power front end of the target clips and of the
style-reference clips (preprocess.py:47-49) -> PerformanceNet forward (model.py:262-300)
-> L1 loss -> backward -> [RCCL gradient all-reduce when N > 1] -> Adam(lr=1e-3)
(train.py:129-143). Dropout on (train mode). Everything inside the timed region runs in
libmst_hip kernels; inputs are resident in HBM before timing starts.

value = (N * 32 * 252) frames / (max over ranks of the timed wall time / K steps).

Launch: python bench.py [--gpus 1] [--steps K] [--warmup W]; N > 1 under
torch.distributed.run (one rank per GPU, RCCL). Rank 0 prints ONE JSON line.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SR = 16000
HOP = 256
T_FRAMES = 252                      # 4.016 s: T = 12 (mod 16) so the U-Net round-trips
L_SAMPLES = HOP * (T_FRAMES - 1)    # 64,256
PEAK_FP32_MFMA = 157.3              # TFLOP/s, MI355X_MICROARCH.md (f32 MFMA = vector rate)
HBM_PEAK_GBS = 8000.0              # GB/s, MI355X_MICROARCH.md (HBM3E)
PEAK_BF16_MFMA = 2500.0             # TFLOP/s dense, MI355X_MICROARCH.md


def synth_clips(n, seed0, L=L_SAMPLES, sr=SR):
    """SURVEY 8(d) synthetic piano clips: Poisson onsets (~4 notes/s), pitch U{21..108},
    duration U[0.1,1] s, velocity U[0.3,1], 8 harmonics 0.6^h, exp(-3t) decay, peak 0.5."""
    clips, notes_all = [], []
    t = np.arange(L) / sr
    for c in range(n):
        rng = np.random.RandomState(seed0 + c)
        dur_total = L / sr
        k = max(1, rng.poisson(4 * dur_total))
        notes = []
        y = np.zeros(L)
        for _ in range(k):
            on = rng.uniform(0, dur_total)
            pitch = rng.randint(21, 109)
            d = rng.uniform(0.1, 1.0)
            vel = rng.uniform(0.3, 1.0)
            f0 = 440.0 * 2 ** ((pitch - 69) / 12)
            tt = t - on
            m = (tt >= 0) & (tt < d + 0.5)
            env = np.exp(-3 * tt[m])
            for h in range(1, 9):
                if h * f0 < sr / 2:
                    y[m] += vel * 0.6 ** h * np.sin(2 * np.pi * h * f0 * tt[m]) * env
            notes.append((pitch, on, min(on + d, dur_total), vel))
        peak = np.abs(y).max()
        clips.append((0.5 * y / peak if peak > 0 else y).astype(np.float32))
        notes_all.append(notes)
    return np.stack(clips), notes_all


def piano_rolls(notes_all, T=T_FRAMES, wps=SR // HOP):
    """pretty_midi-style roll at fs = wps (preprocess.py:147-155), binarised; onoff = diff."""
    rolls = np.zeros((len(notes_all), 128, T), np.float32)
    for i, notes in enumerate(notes_all):
        for p, s, e, _ in notes:
            rolls[i, p, int(s * wps):int(e * wps)] = 1
    prev = np.concatenate([np.zeros_like(rolls[:, :, :1]), rolls[:, :, :-1]], 2)
    return rolls, rolls - prev


def cpu_model():
    """The host CPU's model name (/proc/cpuinfo) for the baseline's record."""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores():
    """(physical cores of the host, logical CPUs) from /proc/cpuinfo."""
    phys, logical = set(), 0
    try:
        with open("/proc/cpuinfo") as fh:
            pid = cid = None
            for line in fh:
                if line.startswith("processor"):
                    logical += 1
                elif line.startswith("physical id"):
                    pid = line.split(":", 1)[1].strip()
                elif line.startswith("core id"):
                    cid = line.split(":", 1)[1].strip()
                    phys.add((pid, cid))
    except OSError:
        pass
    return (len(phys) or None), (logical or os.cpu_count())


def cpu_share():
    """CPU threads this process may use: the runner's per-GPU CPU allotment (OMP_NUM_THREADS:
    16 on the GPU boxes, whose host CPUs are shared by eight GPUs' jobs), capped by the CPUs the
    process is allowed to run on. SURVEY 8(d) asks for all physical cores; on a shared 8-GPU
    host that is the allotment, and the host's own core count is recorded beside it."""
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = os.cpu_count() or 1
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(env, allowed) if env > 0 else allowed)


def cpu_baseline(B=32, steps=1):
    """The oracle's torch-CPU restatement of the reference training step (oracle/model_ref.py),
    timed on this host at the benchmarked configuration (B=32, T=252): `steps` timed steps after
    one untimed warm-up step (fwd + L1 + bwd + Adam, dropout on), on every CPU thread of this
    job's allotment (cpu_share)."""
    from oracle import model_ref as R
    from oracle import detinit
    threads = cpu_share()
    torch.set_num_threads(threads)
    p = R.det_params()
    for v in p.values():
        v.requires_grad_(True)
    xm, xa, cd, tg = (torch.from_numpy(a) for a in detinit.model_inputs(B, T_FRAMES))
    state = {}

    def step(i):
        for v in p.values():
            v.grad = None
        y = R.forward(p, xm, xa, cd, train=True)
        loss = R.l1_loss(y, tg)
        loss.backward()
        with torch.no_grad():
            R.adam_step(p, {k: v.grad for k, v in p.items() if not k.startswith("MBR")}, state, i + 1)
        return loss.item()

    step(0)
    t0 = time.perf_counter()
    for i in range(steps):
        step(i + 1)
    dt = (time.perf_counter() - t0) / steps
    phys, logical = host_cores()
    return {"value": round(B * T_FRAMES / dt, 2), "unit": "spectrogram-frames/s", "cores": threads,
            "kind": "port", "cpu_model": cpu_model(), "host_physical_cores": phys,
            "host_logical_cpus": logical,
            "cores_basis": "the job's CPU allotment (OMP_NUM_THREADS, affinity), all of it used",
            "sample": f"{steps} timed train step(s) (fwd+L1+bwd+Adam, dropout on) of "
                      f"oracle/model_ref.py on torch-CPU after 1 warm-up step, B={B}, T={T_FRAMES} "
                      f"(the benchmarked configuration), {threads} threads ({dt:.2f} s/step)"}


def gemm_traffic():
    """HBM-side bytes per GEMM launch (gemm_kernel and gemm_w_kernel) from this round's PMC passes (tools/pmc_traffic.py
    over `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` runs of this bench), newest round
    first. Returns (bytes or None, source note)."""
    pdir = os.path.join(ROOT, "profiles")
    rounds = sorted((d for d in os.listdir(pdir) if d.startswith("r")), reverse=True) \
        if os.path.isdir(pdir) else []
    for r in rounds:
        tj = os.path.join(pdir, r, "gemm_traffic.json")
        if os.path.exists(tj):
            with open(tj) as fh:
                d = json.load(fh)
            return round(d["traffic_bytes_per_launch"]), (
                f"profiles/{r}/gemm_traffic.json ({d.get('build', 'build not recorded')}): "
                "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes over this bench, "
                "2 x fetch + write per GEMM launch")
    return None, None


def gemm_pmc():
    """MFMA-busy and VALU:MFMA per GEMM kind from the newest round's committed PMC summary
    (profiles/r*/gemm_pmc.json: tools/pmc_gemm_json.py over rocprofv3 --pmc passes of this bench)."""
    pdir = os.path.join(ROOT, "profiles")
    rounds = sorted((d for d in os.listdir(pdir) if d.startswith("r")), reverse=True) \
        if os.path.isdir(pdir) else []
    for r in rounds:
        pj = os.path.join(pdir, r, "gemm_pmc.json")
        if os.path.exists(pj):
            with open(pj) as fh:
                d = json.load(fh)
            return {"build": d.get("build"), "source": f"profiles/{r}/gemm_pmc.json",
                    "kinds": {k: {x: y for x, y in e.items() if x != "counters"}
                              for k, e in d.get("kinds", {}).items()}}
    return None


def aux_legs(world, rank, dev, cpu):
    """BASELINE configs[1] (STFT/mel + 60-iteration Griffin-Lim, 256 x 4 s @ 16 kHz) and
    configs[4] (multi-scale spectral loss, 10 s @ 22.05 kHz) timed in the same run as the
    training step (bench_aux.py's legs, shortened; one-thread oracle CPU baselines)."""
    import bench_aux
    a = argparse.Namespace(steps=10, warmup=2, clips=256, pairs=32, no_cpu_baseline=not cpu,
                           parallel_cpu=True, no_parity=False, strict=False)
    out = {}
    for fn in (bench_aux.frontend, bench_aux.griffinlim, bench_aux.mss):
        for ln in fn(a, world, rank, dev):
            key = ln["config"]["workload"]
            out[key] = {k: ln[k] for k in ("metric", "value", "unit", "ms_per_step", "kernel_ms",
                                           "roofline", "cpu_baseline", "parity") if k in ln}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-timing-steps", type=int, default=2)
    ap.add_argument("--no-aux", action="store_true",
                    help="skip the config-2 / config-5 legs (STFT, mel, Griffin-Lim, multi-scale loss)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="all-reduce after backward instead of overlapped bucket all-reduces")
    ap.add_argument("--graph", action="store_true",
                    help="N=1: replay forward + L1 + backward + Adam as one captured hipGraph "
                         "(graphs.GraphedTrainStep); the STFT front end stays eager")
    ap.add_argument("--adam-overlap", action="store_true",
                    help="(the default since round 5) Adam per bucket inside backward on a side "
                         "stream (train.BackwardAdam), as train.main runs it")
    ap.add_argument("--adam-step", action="store_true",
                    help="Adam as one launch in opt.step() instead (the pre-round-5 default)")
    ap.add_argument("--loss", default="l1", choices=["l1", "mss", "l1+mss"],
                    help="training loss: train.py:132's L1 (the headline), the README's multi-scale "
                         "spectral loss on audio rendered with the target's phase, or both")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if os.environ.get("MST_BENCH_BACKEND", "nccl") != "nccl":
        local_rank %= torch.cuda.device_count()  # rehearsal: ranks may share a GPU
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # MST_BENCH_BACKEND=gloo rehearses the N>1 path with ranks sharing one GPU (RCCL needs
        # one GPU per rank); measured runs use nccl (= RCCL over xGMI)
        backend = os.environ.get("MST_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from ml_music_style_transfer_amd import dp, spectral
    from ml_music_style_transfer_amd import engine as E
    from ml_music_style_transfer_amd import kernels as K
    from ml_music_style_transfer_amd.model import PerformanceNet
    from ml_music_style_transfer_amd.train import make_optimizer

    B = args.batch
    torch.manual_seed(1234)
    model = PerformanceNet().to(dev)
    model.train()
    model._seed += rank << 24  # per-rank dropout streams (train.main does the same)
    dp.broadcast_parameters(model)
    if world > 1 and not args.no_overlap:
        dp.enable_overlapped_allreduce(model)
    # Adam runs bucket by bucket inside backward on its own stream (train.BackwardAdam, bitwise
    # the one-launch update; train.main does the same): since round 5's stream changes it beats
    # the one launch in opt.step() by 1.5-2.3 % per step (profiles/r05/ab_step_adam_overlap_final
    # .jsonl). --adam-step restores the one launch (and the in-step Adam timing leg).
    adam_overlap = not args.adam_step and not args.graph
    opt = make_optimizer(model, lr=1e-3, overlap_backward=adam_overlap and not args.no_overlap)
    if os.environ.get("MST_BENCH_PREALLOC", "0") == "1":  # A/B: Adam moments allocated up front
        opt.prepare()

    # synthetic per-rank data, resident in HBM: target clips, style-reference clips, rolls
    tgt_audio, notes = synth_clips(B, 1234 + 1000 * rank)
    ref_audio, _ = synth_clips(B, 777_000 + 1000 * rank)
    roll, onoff = piano_rolls(notes)
    tgt_audio = torch.from_numpy(tgt_audio).to(dev)
    ref_audio = torch.from_numpy(ref_audio).to(dev)
    data = torch.from_numpy(np.concatenate([roll, onoff], 1)).to(dev)  # (B, 256, T) train.py:84-85

    comm_on = [True]  # off only for the exposed-communication leg after the timed region
    gstep = None
    if args.graph:
        if world > 1 or args.loss != "l1":
            raise SystemExit("--graph: single GPU, L1 loss")
        from ml_music_style_transfer_amd.graphs import GraphedTrainStep
        gstep = GraphedTrainStep(model, opt, warmup=1)

    graph_on = [True]  # off for the per-launch GEMM timing leg (a replay runs no Python)
    adam_ev = []       # HIP events around opt.step() in the timed steps (the adam_kernel leg)
    adam_on = [False]

    def loss_of(y, target, which):
        if which == "l1":
            return E.l1_loss(y, target)
        # the README's loss (README.md:23) on audio rendered from the prediction with the target
        # clip's STFT phase; the target waveform is the clip itself
        mss = spectral.spectrogram_mss_loss(y, tgt_audio, phase="target", hop=HOP)
        return mss if which == "mss" else E.l1_loss(y, target) + mss

    def step(which=None):
        which = which or args.loss
        if gstep is not None and graph_on[0]:
            target = spectral.stft_logpow(tgt_audio, hop=HOP)
            x_audio = spectral.stft_logpow(ref_audio, hop=HOP)
            split = torch.split(data, 128, dim=1)
            return gstep(split[0], x_audio, split[1], target)
        opt.zero_grad()
        target = spectral.stft_logpow(tgt_audio, hop=HOP)           # (B, 1025, 252)
        x_audio = spectral.stft_logpow(ref_audio, hop=HOP)          # style reference spec
        split = torch.split(data, 128, dim=1)                      # train.py:130
        y = model(split[0], x_audio, split[1])
        loss = loss_of(y, target, which)
        loss.backward()               # overlapped bucket all-reduces start inside backward
        if world > 1 and args.no_overlap and comm_on[0]:
            dp.allreduce_gradients(model)
        if adam_on[0]:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        opt.step()                    # waits for the all-reduce, then the update (or joins it)
        if adam_on[0]:
            ev[1].record()
            adam_ev.append(ev)
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    adam_on[0] = gstep is None and not adam_overlap
    for _ in range(args.steps):
        loss = step()
    adam_on[0] = False
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], device=dev)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        dt = tt.item()
    ms_per_step = 1000.0 * dt / args.steps
    value = world * B * T_FRAMES / (dt / args.steps)
    final_loss = loss.item()
    if not math.isfinite(final_loss):
        raise SystemExit(f"non-finite training loss {final_loss}: the measured step is broken")

    # roofline leg: per-launch HIP events around every GEMM (fp32 MFMA implicit GEMM) of a few
    # extra steps, on the launch stream; achieved = algorithmic FLOPs / summed kernel time.
    log = []
    graph_on[0] = False
    from ml_music_style_transfer_amd import model as model_mod
    wgrad_side, enc_side = model_mod._WGRAD_STREAM, model_mod._ENC_STREAM
    model_mod.set_wgrad_stream(False)  # per-launch times need the GEMMs serialised
    model_mod.set_enc_stream(False)
    bwd_adam = getattr(opt, "_bwd", None)
    if bwd_adam is not None:
        bwd_adam.paused = True  # no Adam stream beside the timed GEMMs either
    K.gemm_timing(log)
    for _ in range(args.kernel_timing_steps):
        step()
    K.gemm_timing(None)
    model_mod.set_wgrad_stream(wgrad_side)
    model_mod.set_enc_stream(enc_side)
    if bwd_adam is not None:
        bwd_adam.paused = False
    torch.cuda.synchronize()
    gemm_ms = sum(ev[0].elapsed_time(ev[1]) for ev in log)
    gemm_flops = sum(ev[2] for ev in log)
    n_steps_t = max(1, args.kernel_timing_steps)
    achieved = gemm_flops / (gemm_ms * 1e-3) / 1e12 if gemm_ms > 0 else 0.0
    # algorithmic bytes per GEMM launch: each operand and the output once, (MK + KN + MN) x 4
    alg_bytes = [4.0 * (shp[0] * shp[2] + shp[2] * shp[1] + shp[0] * shp[1]) for *_, shp in log if shp]
    traffic, traffic_src = gemm_traffic()
    # the GEMMs' arithmetic: fp32 products on the bf16 matrix cores (bf16x6 exact split, six
    # bf16 products each) or the fp32 MFMA. The roofline peak is the dense MFMA peak for the
    # path's dtype (f32: 157.3 TF/s); the split build's own ceiling (bf16 peak / 6) rides beside it
    from ml_music_style_transfer_amd import _lib
    products = int(_lib.load().mst_gemm_products())
    # the ceiling of the instructions the GEMMs actually run: bf16 dense MFMA peak / products per
    # fp32 multiply-add (416.7 TF/s of fp32 products for bf16x6); fp32 MFMA for a 1-product build
    split_peak = PEAK_BF16_MFMA / products if products > 1 else None
    peak = split_peak if split_peak else PEAK_FP32_MFMA
    by_tag = {}
    for s, e, f, tag, _ in log:
        a = by_tag.setdefault(tag, [0.0, 0.0, 0])
        a[0] += s.elapsed_time(e)
        a[1] += f
        a[2] += 1

    comm = None
    if world > 1:
        try:
            comm = all_reduce_leg(model, step, comm_on, world, dev, ms_per_step, args)
        except Exception as e:  # a report leg must not cost the measured line
            comm = {"error": repr(e)[:200]}

    out = {
        "metric": "training-step spectrogram-frames/sec, batch 32, 4 s @ 16 kHz, 1/2/4/8 GPUs",
        "value": round(value, 1),
        "unit": "spectrogram-frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (16 kHz piano clips per SURVEY 8(d); random-init PerformanceNet weights)",
        "config": {"workload": "PerformanceNet train step: STFT front end + fwd + "
                               + {"l1": "L1", "mss": "multi-scale spectral loss (rendered audio)",
                                  "l1+mss": "L1 + multi-scale spectral loss"}[args.loss] + " + bwd"
                               + (" + RCCL all-reduce" if world > 1 else "") + " + Adam",
                   "loss": args.loss,
                   "global_batch": world * B, "batch_per_gpu": B, "seq_len": T_FRAMES,
                   "sample_rate": SR, "n_fft": 2048, "hop": HOP, "parallelism": f"dp{world}"},
        "roofline": {
            "bound": "mfma",
            "kernel": ("gemm_w_kernel (128 x 256 tiles: conv/linear fwd and dgrad, operands split in "
                       "registers) and gemm_p_kernel (128 x 256: wgrad on operand planes pre-split by "
                       "pack_planes_kernel, LDS-DMA, the second wave per SIMD staggered, split-K) "
                       "(implicit GEMM; fp32 operands "
                       + ("split into 3 bf16 pieces, 6 x v_mfma_f32_32x32x16_bf16 per 16-deep k step)"
                          if products > 1 else "v_mfma_f32_32x32x2_f32)")),
            "achieved": round(achieved, 2),
            "peak": round(peak, 1),
            "peak_basis": (f"hardware ceiling of the instructions run: bf16 dense MFMA {PEAK_BF16_MFMA:g} "
                           f"TF/s / {products} bf16 products per fp32 multiply-add; achieved counts "
                           "fp32 multiply-adds (2 M N K per GEMM)" if split_peak else
                           "dense fp32 MFMA peak; achieved counts fp32 multiply-adds"),
            "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4),
            "frac_basis": ("achieved / peak, peak = the instruction ceiling above (since round 5); "
                           "rounds 1-4 reported frac against the fp32 MFMA peak, which is "
                           "frac_of_fp32_mfma_peak here: compare across rounds on that field"),
            "fp32_mfma_peak": PEAK_FP32_MFMA,
            "frac_of_fp32_mfma_peak": round(achieved / PEAK_FP32_MFMA, 4),
            "fp32_mfma_peak_basis": ("what an fp32 user gets against the chip's fp32 MFMA rate "
                                     "(the same arithmetic; not a hardware fraction of this build)"),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": round(sum(alg_bytes) / max(len(alg_bytes), 1)),
            "gemm_gflop_per_step": round(gemm_flops / n_steps_t / 1e9, 1),
            "gemm_ms_per_step": round(gemm_ms / n_steps_t, 3),
            "launches_per_step": len(log) // n_steps_t,
            "avg_launch_ms": round(gemm_ms / max(len(log), 1), 4),
            "by_kind": {k: {"ms_per_step": round(v[0] / n_steps_t, 3),
                            "tflops": round(v[1] / (v[0] * 1e-3) / 1e12, 2) if v[0] else 0,
                            "frac": round(v[1] / (v[0] * 1e-3) / 1e12 / peak, 4) if v[0] else 0}
                        for k, v in by_tag.items()},
            "pmc": gemm_pmc(),
            "dvfs": {
                "note": ("the chip holds 1.79-2.09 GHz (not 2.4) in these MFMA-dense loops on random "
                         "data: in-kernel s_memtime / s_memrealtime of the planes GEMM on the step's "
                         "shapes (MI355X_MICROARCH.md, DVFS give-back). The instruction ceiling at that "
                         "clock is 416.7 x clock / 2.4"),
                "clock_GHz": [1.79, 2.09],
                "ceiling_at_clock_TFps": [310.2, 362.9],
                "source": "profiles/r06/gemm_planes_micro_stagger.txt (tools/micro/gemm_planes.hip v8/v10)",
            },
        },
        "final_loss": round(final_loss, 5),
    }
    adam_note = "the optimizer step of the timed steps"
    if not adam_ev and adam_overlap and opt._flat_groups and gstep is None:
        # the timed steps ran Adam per bucket inside backward: time the same kernel over the whole
        # flat buffer in isolation, after every measured leg above (one more update of the state)
        pf, gf, _ = model.flat_buffers()
        st = next(iter(opt._flat_groups.values()))
        evs = []
        for _ in range(4):
            e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            e[0].record()
            K.adam(pf, gf, st["m"], st["v"], 1e-3, 0.9, 0.999, 1e-8, 1.0)
            e[1].record()
            evs.append(e)
        torch.cuda.synchronize()
        adam_ev = evs[1:]
        adam_note = ("measured in isolation after the timed region (the timed steps run it per "
                     "bucket inside backward, train.BackwardAdam)")
    if adam_ev:
        # one adam_kernel over the flat buffer, 28 B per parameter: p, m, v read + written, g
        # read; HIP events on its launch stream
        n_par = int(model.flat_buffers()[2])  # the flat buffer the kernel streams (the dead MBR
        # convolutions' weights are not in it)
        a_ms = sum(e0.elapsed_time(e1) for e0, e1 in adam_ev) / len(adam_ev)
        a_gbs = 28.0 * n_par / (a_ms * 1e-3) / 1e9
        out["adam"] = {"kernel": "adam_kernel (flat fp32 p/g/m/v, torch.optim.Adam arithmetic)",
                       "timing": adam_note, "inside_backward": bool(adam_overlap),
                       "bound": "hbm", "params": n_par, "bytes_per_step": 28 * n_par,
                       "ms_per_step": round(a_ms, 3), "achieved": round(a_gbs, 1),
                       "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(a_gbs / HBM_PEAK_GBS, 4)}
    if comm is not None:
        out["allreduce"] = comm
    if gstep is not None:
        out["config"]["hipgraph"] = True
    if not args.no_aux:
        out["aux"] = aux_legs(world, rank, dev, cpu=not args.no_cpu_baseline)
        if args.loss == "l1" and gstep is None:
            try:  # the same step with the README's loss (after the timed region)
                out["aux"]["train_step_mss"] = mss_step_leg(step, world, dev, B, args)
            except Exception as e:  # a report leg must not cost the measured line
                out["aux"]["train_step_mss"] = {"error": repr(e)[:200]}
        try:  # reference inference call (inference.py:74-91): B = 1, one 4 s chunk
            from ml_music_style_transfer_amd.graphs import inference_step_times
            out["aux"]["inference_b1"] = {k: (round(v, 4) if isinstance(v, float) else v)
                                          for k, v in inference_step_times(model).items()}
        except Exception as e:  # a report leg must not cost the measured line
            out["aux"]["inference_b1"] = {"error": repr(e)[:200]}
    if rank == 0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline()
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


def mss_step_leg(step, world, dev, B, args, reps=5):
    """The benchmarked step with the multi-scale spectral loss as the training loss (L1 + MSS on
    audio rendered with the target's phase: train.make_loss's 'l1+mss' with the bench's own target
    clips), timed like the headline (barrier + synchronize brackets, max over ranks)."""
    for _ in range(2):
        step("l1+mss")
    torch.cuda.synchronize()
    if world > 1:
        dt = _timed_max(lambda: step("l1+mss"), reps, dev)
    else:
        t0 = time.perf_counter()
        for _ in range(reps):
            step("l1+mss")
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    ms = 1000.0 * dt / reps
    return {"metric": "training-step spectrogram-frames/sec with L1 + multi-scale spectral loss",
            "value": round(world * B * T_FRAMES / (dt / reps), 1), "unit": "spectrogram-frames/s",
            "ms_per_step": round(ms, 3), "steps": reps, "loss": "l1+mss",
            "workload": "the headline step, loss = L1 + spectral.spectrogram_mss_loss(phase='target') "
                        "(render kernel, iSTFT + adjoint, 6-size loss kernels)"}


def _timed_max(fn, reps, dev):
    """Wall time of `reps` calls between barrier + synchronize brackets, max over ranks."""
    torch.cuda.synchronize()
    torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    torch.distributed.barrier()
    torch.cuda.synchronize()
    tt = torch.tensor([time.perf_counter() - t0], device=dev)
    torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
    return tt.item()


def all_reduce_leg(model, step, comm_on, world, dev, ms_per_step, args):
    """SURVEY 8(d) config 4, measured after the timed region (the weights diverge here, nothing
    after it trains): (1) the same step with the gradient exchange switched off, so exposed
    communication = ms_per_step - compute-only ms; (2) the bucketed gradient all-reduce alone,
    bus bandwidth = 2 (N-1)/N x bytes / time (RCCL's busbw convention)."""
    from ml_music_style_transfer_amd import dp
    saved = getattr(model, "_mst_dp", None)
    model._mst_dp, comm_on[0] = None, False
    step()
    k = max(2, min(args.steps, 5))
    compute_ms = 1000.0 * _timed_max(step, k, dev) / k
    model._mst_dp, comm_on[0] = saved, True
    _, _, n = model.flat_buffers()
    nbytes = 4 * n
    dp.allreduce_gradients(model, bucket_bytes=dp.OVERLAP_BUCKET_BYTES)
    reps = 3
    t_ar = _timed_max(lambda: dp.allreduce_gradients(model, bucket_bytes=dp.OVERLAP_BUCKET_BYTES),
                      reps, dev) / reps
    return {"grad_bytes": nbytes, "bucket_bytes": dp.OVERLAP_BUCKET_BYTES,
            "allreduce_ms": round(1000.0 * t_ar, 3),
            "bus_GBps": round(2.0 * (world - 1) / world * nbytes / t_ar / 1e9, 1),
            "compute_only_ms_per_step": round(compute_ms, 3),
            "exposed_comm_ms_per_step": round(ms_per_step - compute_ms, 3),
            "overlapped": not args.no_overlap}


if __name__ == "__main__":
    main()
