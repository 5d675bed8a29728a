"""Secondary measurements (not the driver's bench line): BASELINE.json configs[1] and [4].

  frontend    config 2: batched STFT log-power and 128-mel of 256 x 4 s @ 16 kHz clips
              (preprocess.py:47-49, tests/plot_spec.py:20). HBM roofline: algorithmic bytes per
              clip 4 L + 4 F T (log-power) and 4 L + 4 M T (mel).
  griffinlim  config 2: 60-iteration Griffin-Lim of the same 256 spectrograms (inference.py:105-110).
              Algorithmic bytes per iteration per clip 28 F T + 8 L.
  mss         config 5: multi-scale spectral loss (6 FFT sizes) forward + gradient on
              10 s @ 22.05 kHz clip pairs (pred = target + 0.05 N(0,1), seed 7). Algorithmic
              bytes per clip pair 6 x 5 x 4 L (SURVEY 8(d)'s per-size streaming model; the fused
              kernel moves 12 B per sample once, so `frac` may exceed 1).

Each workload prints one JSON line with the same fields as bench.py (value = whole-job
throughput with inputs resident in HBM; kernel time by HIP events on the launch stream) and
a cpu_baseline from the oracle on a bounded sample. N > 1 under torch.distributed.run shards
clips across ranks (independent units, no collective).

usage: python bench_aux.py [--workload frontend|griffinlim|mss|all] [--steps K] [--warmup W]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (synthetic clip recipe)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E ~8 TB/s


def _dist():
    """One process per GPU under torch.distributed.run; every rank takes its own clips (seeded by
    rank, no collective on the data path), barriers + a MAX of the wall time bracket the timing.
    MST_BENCH_BACKEND=gloo rehearses it with ranks sharing one GPU (not an xGMI measurement)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("MST_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    return world, rank, dev


def _timed(fn, steps, warmup, world):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], device=torch.cuda.current_device())
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        dt = tt.item()
    return dt / steps


def _event_ms(fn, reps=5):
    """Average duration of fn's launches, HIP events on the current (launch) stream."""
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def _measured_traffic(kernel_key):
    """HBM bytes per launch of a kernel from the newest round's PMC passes (tools/pmc_traffic.py:
    2 x FETCH_SIZE + WRITE_SIZE over `rocprofv3 --pmc` runs of this script), or (None, None)."""
    pdir = os.path.join(ROOT, "profiles")
    for r in sorted((d for d in os.listdir(pdir) if d.startswith("r")), reverse=True) if os.path.isdir(pdir) else []:
        tj = os.path.join(pdir, r, "stft_traffic.json")
        if os.path.exists(tj):
            d = json.load(open(tj))
            for k, v in d.get("per_kernel", {}).items():
                if kernel_key in k:
                    return round(2 * v["fetch_raw_per_launch"] + v["write_per_launch"]), \
                        f"profiles/{r}/stft_traffic.json ({d.get('build', '')})"
    return None, None


def _gl_traffic(n_iter):
    """HBM bytes of one Griffin-Lim call from the newest round's PMC passes over the Griffin-Lim
    leg (profiles/r*/gl_traffic.json): (n_iter + 1) syntheses (+ seam passes in earlier builds), n_iter complex
    STFTs and the one magnitude transpose, each 2 x FETCH_SIZE + WRITE_SIZE per launch."""
    pdir = os.path.join(ROOT, "profiles")
    for r in sorted((d for d in os.listdir(pdir) if d.startswith("r")), reverse=True) if os.path.isdir(pdir) else []:
        tj = os.path.join(pdir, r, "gl_traffic.json")
        if not os.path.exists(tj):
            continue
        d = json.load(open(tj))
        per = {}
        for k, v in d.get("per_kernel", {}).items():
            # the complex STFT: stft_fm_kernel<3, ...> (late round 2) or stft_kernel<3> (before)
            for key, name in (("gl_synth_kernel", "synth"), ("gl_seam_kernel", "seam"), ("stft_kernel<3>", "cx"),
                              ("stft_fm_kernel<3,", "cx"), ("transpose_mag_kernel", "tmag"),
                              ("fillBufferAligned", "memset")):
                if key in k:
                    per[name] = 2 * v["fetch_raw_per_launch"] + v["write_per_launch"]
        if "synth" not in per or "cx" not in per:
            continue
        tot = ((n_iter + 1) * (per["synth"] + per.get("seam", 0.0))
               + n_iter * per["cx"] + per.get("tmag", 0.0)
               + per.get("memset", 0.0))  # the seam-zeroing memset (atomic-seam builds)
        return round(tot), f"profiles/{r}/gl_traffic.json ({d.get('build', '')})"
    return None, None


def _mss_traffic():
    """HBM bytes of one multi-scale loss call (six size kernels + edge fold + loss reduce) from the
    newest round's PMC passes over the loss leg (profiles/r*/mss_traffic.json)."""
    pdir = os.path.join(ROOT, "profiles")
    for r in sorted((d for d in os.listdir(pdir) if d.startswith("r")), reverse=True) if os.path.isdir(pdir) else []:
        tj = os.path.join(pdir, r, "mss_traffic.json")
        if not os.path.exists(tj):
            continue
        d = json.load(open(tj))
        tot = sum(2 * v["fetch_raw_per_launch"] + v["write_per_launch"]
                  for k, v in d.get("per_kernel", {}).items() if "mss_" in k)
        return round(tot), f"profiles/{r}/mss_traffic.json ({d.get('build', '')})"
    return None, None


def _roof(achieved_gbs, kernel, bytes_per_launch, traffic_key=None, traffic=None):
    if traffic is not None:
        traffic, src = traffic
    else:
        traffic, src = _measured_traffic(traffic_key) if traffic_key else (None, None)
    out = {"bound": "hbm", "kernel": kernel, "achieved": round(achieved_gbs, 1),
           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
           "traffic": traffic, "algorithmic_bytes_per_launch": int(bytes_per_launch)}
    if src:
        out["traffic_source"] = src
    return out


def _line(metric, value, unit, world, steps, warmup, ms, config, roofline, cpu, extra=None):
    out = {"metric": metric, "value": round(value, 2), "unit": unit, "n_gpus": world,
           "steps": steps, "warmup": warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
           "config": config, "roofline": roofline}
    if cpu is not None:
        out["cpu_baseline"] = cpu
    if extra:
        out.update(extra)
    return out


def _cpu_front(job):
    """One clip through the oracle (runs in a spawned worker: NumPy only, no GPU)."""
    from oracle import spectral_ref as SR
    name, clip = job
    return (SR.logpow(clip, 2048, bench.HOP) if name == "logpow"
            else SR.melspec(clip, bench.SR, 2048, bench.HOP)).shape


def _cpu_gl(job):
    """One clip x n_iter Griffin-Lim iterations through the oracle (spawned worker, NumPy only)."""
    from oracle import spectral_ref as SR
    clip, n_iter = job
    Sn = np.abs(SR.stft(clip, 2048, bench.HOP, out_dtype=None))
    SR.griffinlim(Sn, n_iter=n_iter, hop=bench.HOP, angles=np.ones_like(Sn, dtype=np.complex128))
    return n_iter


def _cpu_mss(job):
    """One clip pair's multi-scale loss + gradient through the oracle (spawned worker)."""
    from oracle import spectral_ref as SR
    p, t, sizes = job
    SR.multiscale_spectral_loss_grad(p, t, 1.0, 1e-7, sizes)
    return 1


def _pool_rate(fn, jobs, warm):
    """Jobs per second over a process pool of the job's CPU allotment (bench.cpu_share; spawned
    workers, one BLAS thread each, no GPU state); pool start-up and a warm-up job per worker are
    outside the timing. Returns (jobs/s, workers)."""
    import multiprocessing as mp
    procs = bench.cpu_share()
    keys = ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")
    saved = {k: os.environ.get(k) for k in keys}
    os.environ.update({k: "1" for k in keys})  # one BLAS thread per worker: no oversubscription
    try:
        pool = mp.get_context("spawn").Pool(procs)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    with pool:
        pool.map(fn, [warm] * procs)  # warm every worker
        t0 = time.perf_counter()
        pool.map(fn, jobs, chunksize=max(1, len(jobs) // (4 * procs)))
        dt = time.perf_counter() - t0
    return len(jobs) / dt, procs


def _cpu_parallel_rate(name, clips):
    """NumPy's FFT is single-threaded, so the n-way CPU number is a process pool
    (spawned workers, no GPU state) over the clips; pool start-up is outside the timing."""
    rate, procs = _pool_rate(_cpu_front, [(name, c) for c in clips], (name, clips[0]))
    return {"value": round(rate, 2), "cores": procs,
            "sample": f"{len(clips)} clips, multiprocessing pool of {procs} spawned workers"}


def _verdict(ok, msg, args):
    """Outcome of a sampled oracle check: bench_aux.py run on its own stops on a miss
    (--strict, the default); bench.py records it in the leg's "parity" object instead, so a
    miss is reported in the measured line rather than costing the whole bench."""
    if not ok:
        if getattr(args, "strict", True):
            raise AssertionError(msg)
        print("PARITY MISS: " + msg, file=sys.stderr, flush=True)
    return {"ok": bool(ok)} if ok else {"ok": False, "miss": msg}


def _sampled(B):
    """Clips checked against the oracle after the timed region: one per residue mod 8 (the
    persistent STFT kernel's XCD groups) and the last clip."""
    return sorted({min(B - 1, 9 * r) for r in range(8)} | {B - 1})


def _frontend_parity(name, out, x, args):
    """Sampled clips of the measured output vs oracle/spectral_ref (tolerances of
    tests/test_gpu_config2.py: log-power 1e-4 absolute, mel 1e-4 of the frame's peak)."""
    from oracle import spectral_ref as SR
    worst = 0.0
    idx = _sampled(len(x))
    for b in idx:
        if name == "logpow":
            err = float(np.abs(out[b] - SR.logpow(x[b], 2048, bench.HOP)).max())
            tol = 1e-4
        else:
            ref = SR.melspec(x[b], bench.SR, 2048, bench.HOP)
            err = float((np.abs(out[b] - ref) / (ref.max(axis=0, keepdims=True) + 1e-12)).max())
            tol = 1e-4
        worst = max(worst, err)
    return {"clips": idx, "max_err": worst, "tol": tol,
            **_verdict(worst <= tol, f"{name}: sampled clips differ from the oracle by {worst} > {tol}", args)}


def frontend(args, world, rank, dev):
    from ml_music_style_transfer_amd import spectral
    from oracle import spectral_ref as SR
    B, L, F, M = args.clips, bench.L_SAMPLES, 1025, 128
    T = 1 + L // bench.HOP
    x, _ = bench.synth_clips(B, 4242 + 100_000 * rank)
    xd = torch.from_numpy(x).to(dev)
    res = []
    for name, fn, bpc, kern, tkey in (
            ("logpow", lambda: spectral.stft_logpow(xd, hop=bench.HOP), 4 * L + 4 * F * T,
             "stft_fm_kernel<LOGPOW> (fft.hip)", "stft_fm_kernel<0,"),
            ("mel", lambda: spectral.melspectrogram(xd, bench.SR, hop_length=bench.HOP), 4 * L + 4 * M * T,
             "stft_fm_kernel<MEL> (fft.hip)", "stft_fm_kernel<2,")):
        dt = _timed(fn, args.steps, args.warmup, world)
        kms = _event_ms(fn)
        cpu = None
        if rank == 0 and not args.no_cpu_baseline:
            n = 16
            t0 = time.perf_counter()
            for i in range(n):
                (SR.logpow(x[i], 2048, bench.HOP) if name == "logpow"
                 else SR.melspec(x[i], bench.SR, 2048, bench.HOP))
            c = (time.perf_counter() - t0) / n
            cpu = {"value": round(1.0 / c, 2), "unit": "clips/s", "cores": 1, "kind": "port",
                   "sample": f"{n} clips through oracle/spectral_ref.py (NumPy pocketfft float64, 1 thread)"}
            if getattr(args, "parallel_cpu", True):
                try:
                    cpu["parallel"] = _cpu_parallel_rate(name, list(x[:min(B, 256)]))
                except Exception as e:  # a baseline leg must not cost the measured line
                    cpu["parallel"] = {"error": repr(e)[:200]}
        extra = {"kernel_ms": round(kms, 4)}
        if rank == 0 and not args.no_parity:
            extra["parity"] = _frontend_parity(name, fn().cpu().numpy(), x, args)
        res.append(_line(f"STFT {name} clips/s, 256 x 4 s @ 16 kHz", world * B / dt, "clips/s", world,
                         args.steps, args.warmup, dt * 1e3,
                         {"workload": f"config 2 front end: {name}", "clips_per_gpu": B, "L": L,
                          "n_fft": 2048, "hop": bench.HOP},
                         _roof(B * bpc / (kms * 1e-3) / 1e9, kern, B * bpc,
                               tkey if B == 256 else None), cpu, extra))
    return res


def _gl_parity(S, y, idx, n_iter, args):
    """Spectral convergence of sampled clips of the measured output vs the oracle's Griffin-Lim
    from the same (all-ones) init: within 2 % (tests/test_gpu_config2.py's bound)."""
    from ml_music_style_transfer_amd import spectral
    from oracle import spectral_ref as SR
    rows, ok, miss = [], True, ""
    for b in idx:
        Sb = S[b].cpu().double().numpy()
        sc = spectral.spectral_convergence(S[b:b + 1], y[b:b + 1], hop=bench.HOP)
        yr = SR.griffinlim(Sb, n_iter=n_iter, hop=bench.HOP)
        sc_ref = float(np.linalg.norm(np.abs(SR.stft(yr, 2048, bench.HOP, out_dtype=None)) - Sb)
                       / np.linalg.norm(Sb))
        if not sc <= sc_ref * 1.02 + 1e-4:
            ok, miss = False, f"Griffin-Lim clip {b}: convergence {sc} vs oracle {sc_ref}"
        rows.append({"clip": b, "spectral_convergence": round(sc, 6), "oracle": round(sc_ref, 6)})
    return {"clips": rows, "tol": "sc <= 1.02 sc_oracle + 1e-4", **_verdict(ok, miss, args)}


def griffinlim(args, world, rank, dev):
    from ml_music_style_transfer_amd import spectral
    from oracle import spectral_ref as SR
    B, L, F = args.clips, bench.L_SAMPLES, 1025
    T = 1 + L // bench.HOP
    x, _ = bench.synth_clips(B, 5151 + 100_000 * rank)
    S = spectral.stft_power(torch.from_numpy(x).to(dev), hop=bench.HOP).clamp_min(0).sqrt()
    n_iter = 60

    def fn():
        return spectral.griffinlim(S, n_iter=n_iter, hop_length=bench.HOP, init=None)

    steps = max(1, args.steps // 4)
    dt = _timed(fn, steps, 1, world)
    kms = _event_ms(fn, reps=2)
    bpi = 28 * F * T + 8 * L
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        Sn = np.abs(SR.stft(x[0], 2048, bench.HOP, out_dtype=None))
        t0 = time.perf_counter()
        SR.griffinlim(Sn, n_iter=10, hop=bench.HOP, angles=np.ones_like(Sn, dtype=np.complex128))
        c = (time.perf_counter() - t0) / 10
        cpu = {"value": round(1.0 / (c * n_iter), 3), "unit": "clips/s (60 iterations)", "cores": 1,
               "kind": "port", "sample": "1 clip x 10 iterations of oracle/spectral_ref.griffinlim "
                                         "(NumPy float64, 1 thread), scaled to 60 iterations"}
        if getattr(args, "parallel_cpu", True):
            try:
                rate, procs = _pool_rate(_cpu_gl, [(x[i], 10) for i in range(bench.cpu_share())], (x[0], 1))
                cpu["parallel"] = {"value": round(rate * 10 / n_iter, 3), "cores": procs,
                                   "sample": f"{procs} clips x 10 iterations, multiprocessing pool of "
                                             f"{procs} spawned workers, scaled to 60 iterations"}
            except Exception as e:  # a baseline leg must not cost the measured line
                cpu["parallel"] = {"error": repr(e)[:200]}
    extra = {"kernel_ms": round(kms, 3)}
    if rank == 0 and not args.no_parity:
        extra["parity"] = _gl_parity(S, fn(), [0, B - 1], n_iter, args)
    return [_line("Griffin-Lim clips/s (60 iterations), 256 x 4 s @ 16 kHz", world * B / dt,
                  "clips/s", world, steps, 1, dt * 1e3,
                  {"workload": "config 2 Griffin-Lim, 60 iterations, momentum 0.99", "clips_per_gpu": B,
                   "L": L, "n_fft": 2048, "hop": bench.HOP},
                  _roof(B * n_iter * bpi / (kms * 1e-3) / 1e9,
                        "gl_synth_kernel (atomic seams) + stft_fm_kernel<COMPLEX> per iteration",
                        B * n_iter * bpi, traffic=_gl_traffic(n_iter)), cpu, extra)]


def _torch_fp32_mss_gap(p, t, sizes, ref):
    """Relative gap of torch's fp32 CPU multi-scale loss (torch.stft) to the float64 oracle."""
    pt, qt, tot = torch.tensor(p), torch.tensor(t), 0.0
    for n in sizes:
        w = torch.hann_window(n, periodic=True)
        a = torch.stft(pt, n, n // 4, window=w, center=True, pad_mode="reflect", return_complex=True).abs()
        b = torch.stft(qt, n, n // 4, window=w, center=True, pad_mode="reflect", return_complex=True).abs()
        tot += ((a - b).abs().mean() + (torch.log(a + 1e-7) - torch.log(b + 1e-7)).abs().mean()).item()
    return abs(tot - ref) / abs(ref)


def mss(args, world, rank, dev):
    from ml_music_style_transfer_amd import spectral
    from oracle import spectral_ref as SR
    B, L = args.pairs, 220_500
    sizes = spectral.MSS_SIZES
    rng = np.random.default_rng(7 + 1000 * rank)
    x, _ = bench.synth_clips(B, 9090 + 100_000 * rank, L=L, sr=22050)
    tgt = torch.from_numpy(x).to(dev)
    pred = (tgt + 0.05 * torch.from_numpy(rng.standard_normal((B, L)).astype(np.float32)).to(dev))
    pred.requires_grad_(True)

    def fn():
        pred.grad = None
        loss = spectral.multiscale_spectral_loss(pred, tgt, sizes=sizes)
        loss.backward()
        return loss

    dt = _timed(fn, args.steps, args.warmup, world)
    kms = _event_ms(fn)
    bpp = len(sizes) * 5 * 4 * L
    flops = sum(3 * 4 * 2.5 * n * np.log2(n) * (1 + L // (n // 4)) / 4 for n in sizes)  # rough
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        p64 = pred.detach()[0].cpu().double().numpy()
        t64 = tgt[0].cpu().double().numpy()
        t0 = time.perf_counter()
        SR.multiscale_spectral_loss_grad(p64, t64, 1.0, 1e-7, sizes)
        c = time.perf_counter() - t0
        cpu = {"value": round(1.0 / c, 3), "unit": "clip-pairs/s", "cores": 1, "kind": "port",
               "sample": "1 clip pair (10 s @ 22.05 kHz), loss + gradient by "
                         "oracle/spectral_ref.multiscale_spectral_loss_grad (NumPy float64)"}
        if getattr(args, "parallel_cpu", True):
            try:
                pr = pred.detach().cpu().double().numpy()
                tg = tgt.cpu().double().numpy()
                n = min(B, bench.cpu_share())
                rate, procs = _pool_rate(_cpu_mss, [(pr[i], tg[i], list(sizes)) for i in range(n)],
                                         (pr[0, :8192], tg[0, :8192], list(sizes)))
                cpu["parallel"] = {"value": round(rate, 3), "cores": procs,
                                   "sample": f"{n} clip pairs, multiprocessing pool of {procs} spawned workers"}
            except Exception as e:  # a baseline leg must not cost the measured line
                cpu["parallel"] = {"error": repr(e)[:200]}
    extra = {"kernel_ms": round(kms, 4), "approx_fft_gflop_per_step": round(B * flops / 1e9, 2)}
    if rank == 0 and not args.no_parity:
        p0 = pred.detach()[:1].clone().requires_grad_(True)
        l0 = spectral.multiscale_spectral_loss(p0, tgt[:1], sizes=sizes)
        ref, _ = SR.multiscale_spectral_loss_grad(p0.detach()[0].cpu().double().numpy(),
                                                  tgt[0].cpu().double().numpy(), 1.0, 1e-7, sizes)
        rel = abs(l0.item() - ref) / abs(ref)
        # north_star's 1e-4 on both input classes. The piano target of pair 0 has exact silence
        # (11 % of its samples) and bins far below fp32 resolution, which log(S + 1e-7)
        # amplifies: torch's own fp32 path misses float64 by 1.2e-3 on it (reported as a
        # diagnostic); the target transform here runs in float64 (mss_target_kernel). The same
        # pair with the silence filled by low-level noise is the non-silent class.
        gap = _torch_fp32_mss_gap(p0.detach()[0].cpu().numpy(), tgt[0].cpu().numpy(), sizes, ref)
        t1 = tgt[:1] + 1e-3 * torch.from_numpy(rng.standard_normal((1, L)).astype(np.float32)).to(dev)
        l1 = spectral.multiscale_spectral_loss(p0.detach(), t1, sizes=sizes)
        ref1, _ = SR.multiscale_spectral_loss_grad(p0.detach()[0].cpu().double().numpy(),
                                                   t1[0].cpu().double().numpy(), 1.0, 1e-7, sizes)
        rel1 = abs(l1.item() - ref1) / abs(ref1)
        ok = rel <= 1e-4 and rel1 <= 1e-4
        extra["parity"] = {"pair": 0, "loss": l0.item(), "oracle": ref, "rel_err": rel,
                           "tol": 1e-4, "torch_fp32_rel_err": gap,
                           "nonsilent": {"loss": l1.item(), "oracle": ref1, "rel_err": rel1, "tol": 1e-4},
                           **_verdict(ok, f"multi-scale loss of pair 0: rel {rel:.2e} (bar 1e-4),"
                                          f" non-silent rel {rel1:.2e} (bar 1e-4)", args)}
    return [_line("multi-scale spectral loss fwd+grad clip-pairs/s, 10 s @ 22.05 kHz, 6 FFT sizes",
                  world * B / dt, "clip-pairs/s", world, args.steps, args.warmup, dt * 1e3,
                  {"workload": "config 5: DDSP multi-scale spectral loss + d/d pred",
                   "pairs_per_gpu": B, "L": L, "sizes": list(sizes)},
                  _roof(B * bpp / (kms * 1e-3) / 1e9,
                        "mss_target_kernel (float64 target magnitudes, every size in one launch), "
                        "mss_multi_kernel (n = 64..1024 in one launch), mss_fft2048_kernel, ordered "
                        "slab sum + fold + loss reduce",
                        B * bpp, traffic=_mss_traffic()), cpu, extra)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="all", choices=["frontend", "griffinlim", "mss", "all"])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--clips", type=int, default=256)
    ap.add_argument("--pairs", type=int, default=32)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-strict", dest="strict", action="store_false",
                    help="record a sampled-check miss in the line instead of stopping")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the sampled-clip oracle check after the timed region")
    args = ap.parse_args()
    world, rank, dev = _dist()
    from ml_music_style_transfer_amd import _lib
    _lib.load()
    lines = []
    for wl, fn in (("frontend", frontend), ("griffinlim", griffinlim), ("mss", mss)):
        if args.workload in (wl, "all"):
            lines += fn(args, world, rank, dev)
    if rank == 0:
        for ln in lines:
            print(json.dumps(ln), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
