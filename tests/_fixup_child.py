"""Child process of tests/test_gpu_kernels.py::test_splitk_fixup_handoff (MST_SPLITK_FIXUP=1 set by
the parent; the library reads it once per process). Split-K reduced inside the 128 x 256 kernels
(gemm.hip splitk_epilogue: slabs stored write-through, per-tile arrival counters, the last arrival
sums the slabs in split order): conv (bias + LeakyReLU epilogue), dgrad and the planes weight
gradient (accumulate) on partial M and N tiles against float64, then 12 launches alternating two
inputs while another stream keeps the GPU busy: every result must be bitwise its input's first
result, so no launch read a stale slab or a stale counter (the counters live in the reused
workspace arena).

usage: MST_SPLITK_FIXUP=1 python tests/_fixup_child.py SPLITK
"""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _r(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(*shape, generator=g, dtype=torch.float64) * 2 - 1


def _close(got, ref, scale, what):
    err = (got.detach().double().cpu() - ref).abs().max().item()
    assert err <= 2e-5 * scale, f"{what}: max err {err:.3e} > {2e-5 * scale:.3e}"


def _conv1d_ref(x, W, b):
    return F.conv1d(x, W, b, padding=1)


def main(splitk, cuda):
    from ml_music_style_transfer_amd import kernels as K
    from ml_music_style_transfer_amd import _lib as L
    B, Cin, Cout, T = 32, 320, 200, 15  # N = 480 (fwd, dgrad), 960 (wgrad): both % 32 == 0
    xs = [_r(B, Cin, T, seed=61 + i) for i in range(2)]
    W, b, dy = _r(Cout, Cin, 3, seed=63), _r(Cout, seed=64), _r(B, Cout, T, seed=65)
    Wd, bd, dyd = W.float().to(cuda), b.float().to(cuda), dy.float().to(cuda)

    def fwd(xd, Wx):
        y = torch.full((B, Cout, T), float("nan"), device=cuda)
        K.conv_like(B=B, M=Cout, Tn=T, srcs=[(xd, 0)], Tv=T, taps=3, a=1, beta=-1, g=1, A=Wx,
                    sAm=Cin * 3, sAc=3, sAt=1, dsts=[(y, 0, None, 1.0)], bias=bd, act=L.ACT_LRELU,
                    splitk=splitk)
        return y

    def wgrad(xd):
        dW = torch.ones(Cout, Cin, 3, device=cuda)
        K.wgrad_like(P=dyd, srcs=[(xd, 0)], Tv=T, taps=3, a=1, beta=-1, g=1, out=dW, ldo=Cin * 3,
                     accumulate=True, splitk=splitk)
        return dW

    def dgrad(Wx):
        dx = torch.full((B, Cin, T), float("nan"), device=cuda)
        K.conv_like(B=B, M=Cin, Tn=T, srcs=[(dyd, 0)], Tv=T, taps=3, a=1, beta=1, g=-1, A=Wx,
                    sAm=Wx.stride(1), sAc=Wx.stride(0), sAt=Wx.stride(2), dsts=[(dx, 0, None, 1.0)],
                    splitk=splitk)
        return dx

    xds = [x.float().to(cuda) for x in xs]
    Ws = [Wd, (Wd * 0.5 + 0.25).contiguous()]
    first = [(fwd(xds[i], Ws[i]), wgrad(xds[i]), dgrad(Ws[i])) for i in range(2)]
    for i in range(2):
        xr = xs[i].clone().requires_grad_(True)
        Wr = (W if i == 0 else W * 0.5 + 0.25).clone().requires_grad_(True)
        yr = _conv1d_ref(xr, Wr, b)
        _close(first[i][0], F.leaky_relu(yr, 0.01).detach(), Cin * 3, what=f"fixup fwd {splitk} input {i}")
        yr.backward(dy)
        Wt = W.clone().requires_grad_(True)
        _conv1d_ref(xs[i], Wt, None).backward(dy)
        _close(first[i][1], 1.0 + Wt.grad, B * T, what=f"fixup wgrad {splitk}")
        _close(first[i][2], xr.grad, Cout * 3, what=f"fixup dgrad {splitk}")
    side = torch.cuda.Stream()
    a = torch.rand(4096, 4096, device=cuda)
    for it in range(12):
        with torch.cuda.stream(side):
            for _ in range(3):
                a = (a @ a).clamp_(-1, 1)
        i = it % 2
        got = (fwd(xds[i], Ws[i]), wgrad(xds[i]), dgrad(Ws[i]))
        for g_, f_, what in zip(got, first[i], ("fwd", "wgrad", "dgrad")):
            assert torch.equal(g_, f_), f"split-K {splitk} launch {it}: {what} differs from its first run"
    torch.cuda.synchronize()
    print("fixup ok")


if __name__ == "__main__":
    main(int(sys.argv[1]), torch.device("cuda"))
