"""Child process of tests/test_gpu_knobs.py: runs a fixed set of kernels under whatever MST_*
environment knobs the parent set (they are read once per process, so each setting needs its own
process) and saves the outputs for the parent to compare against its own default-build results.

usage: python tests/_knob_child.py OUT.npz
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _r(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(*shape, generator=g, dtype=torch.float32) * 2 - 1


def run(dev):
    """Outputs of conv3 fwd/dgrad/wgrad (one shape on the split-K schedule, one without), the
    InstanceNorm forward/backward at segment and full-wave row lengths, Adam, and a short
    Griffin-Lim. Returns {name: numpy array}."""
    from ml_music_style_transfer_amd import kernels as K
    from ml_music_style_transfer_amd import spectral

    out = {}
    for tag, (B, Cin, Cout, T) in {"deep": (32, 512, 512, 15), "wide": (4, 96, 130, 252)}.items():
        x, W, b = _r(B, Cin, T, seed=1).to(dev), _r(Cout, Cin, 3, seed=2).to(dev), _r(Cout, seed=3).to(dev)
        dy = _r(B, Cout, T, seed=4).to(dev)
        y = torch.empty(B, Cout, T, device=dev)
        K.conv3_fwd([(x, 0)], W, b, y)
        dx = torch.empty_like(x)
        K.conv3_dgrad(dy, W, [(dx, 0, None, 1.0)])
        dW = torch.empty_like(W)
        K.conv3_wgrad(dy, [(x, 0)], dW, False)
        out.update({f"{tag}_fwd": y, f"{tag}_dgrad": dx, f"{tag}_wgrad": dW})
    for T in (15, 252):
        yv = _r(3, 7, T, seed=5).to(dev) * 3 + 0.5
        a, pooled, mean, rstd = K.in_lrelu_fwd(yv, True)
        da, dp = _r(3, 7, T, seed=6).to(dev), _r(3, 7, T // 2, seed=7).to(dev)
        dyv, rs = K.in_lrelu_bwd(yv, mean, rstd, da, dp, None, rowsum=True)
        out.update({f"in{T}_a": a, f"in{T}_pool": pooled, f"in{T}_dy": dyv, f"in{T}_rs": rs})
    n = 100_003
    w = _r(n, seed=8).to(dev)
    m, v = torch.zeros_like(w), torch.zeros_like(w)
    for step in range(1, 3):
        K.adam(w, _r(n, seed=10 + step).to(dev), m, v, 1e-3 / (1 - 0.9 ** step), 0.9, 0.999, 1e-8,
               (1 - 0.999 ** step) ** 0.5)
    out["adam_w"] = w
    S = (_r(2, 1025, 40, seed=9).abs() + 0.1).to(dev)
    out["gl"] = spectral.griffinlim(S, n_iter=3, hop_length=256, seed=3)
    torch.cuda.synchronize()
    return {k: t.detach().float().cpu().numpy() for k, t in out.items()}


if __name__ == "__main__":
    np.savez(sys.argv[1], **run(torch.device("cuda")))
