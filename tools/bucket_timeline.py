"""When each gradient bucket of the data-parallel all-reduce becomes ready inside backward (dev tool).

One GPU, the bench's training step (B = 32, T = 252, train mode, the default streams). A stand-in
for dp.OverlappedAllReduce is attached: the same 128 MB buckets and the same issue rule (a bucket is
issued once every parameter in it is done, in order, from the stream the block listeners run on),
but instead of the RCCL all-reduce it records a HIP event there. The events give each bucket's
ready time relative to the start of backward, and the end of backward (the compute stream's last
kernel before Adam). From that timeline a serial communication stream is simulated for N = 8 at a
range of all-reduce bus bandwidths (ring: 2 (N - 1) / N x bucket bytes / bus bandwidth per bucket):
the exposed communication is what runs past the end of backward.

usage (GPU box): python tools/bucket_timeline.py [--steps 3] > profiles/r06/bucket_timeline.txt
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--world", type=int, default=8)
    args = ap.parse_args()
    import bench
    from ml_music_style_transfer_amd import dp
    from ml_music_style_transfer_amd import engine as E
    from ml_music_style_transfer_amd import spectral
    from ml_music_style_transfer_amd.model import PerformanceNet
    from ml_music_style_transfer_amd.train import make_optimizer

    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    model = PerformanceNet().to(dev).train()

    class Probe(dp.OverlappedAllReduce):
        def begin(self):
            self.remaining = list(self.count)
            self.next = 0
            self.works = []
            self.scaled = []
            self.active = True
            self.events = []

        def _launch(self, b):
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()  # on the stream the listeners issue from (the weight-gradient stream)
            self.events.append(ev)

        def finish(self):
            self.launch_remaining()
            self.active = False

    probe = Probe(model)
    model._mst_dp = probe
    opt = make_optimizer(model, lr=1e-3)
    B = args.batch
    tgt, notes = bench.synth_clips(B, 1234)
    ref, _ = bench.synth_clips(B, 777_000)
    roll, onoff = bench.piano_rolls(notes)
    import numpy as np
    tgt, ref = torch.from_numpy(tgt).to(dev), torch.from_numpy(ref).to(dev)
    data = torch.from_numpy(np.concatenate([roll, onoff], 1)).to(dev)
    rows = []
    for it in range(args.steps + 1):
        opt.zero_grad()
        target = spectral.stft_logpow(tgt, hop=bench.HOP)
        x_audio = spectral.stft_logpow(ref, hop=bench.HOP)
        split = torch.split(data, 128, dim=1)
        y = model(split[0], x_audio, split[1])
        loss = E.l1_loss(y, target)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        loss.backward()
        e1.record()  # the compute stream after backward (it has joined the side streams)
        probe.finish()
        opt.step()
        torch.cuda.synchronize()
        if it == 0:
            continue  # warmup
        rows.append(([e0.elapsed_time(ev) for ev in probe.events], e0.elapsed_time(e1)))
    sizes = [(e - s) * 4 for s, e in probe.buckets]
    ready = [sum(r[0][b] for r in rows) / len(rows) for b in range(len(sizes))]
    bwd = sum(r[1] for r in rows) / len(rows)
    N = args.world
    print(f"# backward {bwd:.2f} ms (B = {B}, T = 252, mean of {len(rows)} steps); "
          f"{len(sizes)} buckets, {sum(sizes) / 1e9:.3f} GB of fp32 gradients")
    print("# bucket  MB   ready_ms (from the start of backward)")
    for b, (sz, t) in enumerate(zip(sizes, ready)):
        print(f"  {b:3d} {sz / 2**20:7.1f} {t:8.2f}")
    print(f"# simulated serial all-reduce stream at N = {N} (ring, 2(N-1)/N x bytes / bus BW per bucket)")
    print("# bus_GBps  comm_ms  comm_end_ms  exposed_ms")
    for bw in (50, 100, 150, 200, 250, 300, 400):
        t = 0.0
        total = 0.0
        for sz, r in zip(sizes, ready):
            d = 2 * (N - 1) / N * sz / (bw * 1e9) * 1e3
            t = max(t, r) + d
            total += d
        print(f"  {bw:8d} {total:8.2f} {t:11.2f} {max(0.0, t - bwd):10.2f}")


if __name__ == "__main__":
    main()
