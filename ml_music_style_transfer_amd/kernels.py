"""Thin tensor-level wrappers over libmst_hip's C ABI (include/mst.h).

Every function enqueues HIP kernels on torch's current stream and returns
without synchronising. Tensors must be contiguous float32 CUDA tensors; there
is deliberately no CPU fallback (see _lib.ptr).

Layer geometry (all implicit GEMMs of gemm.hip; reference model/model.py):
  conv3   nn.Conv1d(k=3, p=1)                       model.py:14-22
  convT2  nn.ConvTranspose1d(k, s=2, p=1)           model.py:24-31   (two sub-pixel phases)
  convT1  nn.ConvTranspose1d(k=3, s=1, p=1)         model.py:242     (lastconv)
  linear  nn.Linear over channels of an NCL tensor  model.py:98-99,104-107
Sources are (tensor, time_offset) pairs forming a virtual channel concat; the
offset implements crop_and_concat (model.py:71-78).
"""
import ctypes
import os

import torch

from . import _lib as L

SLOPE = 0.01
IN_EPS = 1e-5
# dev-only A/B knob: force one K schedule on every GEMM (mst_conv_desc.splitk semantics)
_FORCE_SPLITK = int(os.environ.get("MST_FORCE_SPLITK", "0"))


def _lib():
    return L.load()


def empty(*shape, like=None, device=None):
    dev = like.device if like is not None else device
    return torch.empty(shape, device=dev, dtype=torch.float32)


def _src(spec):
    s = L.MstSrc()
    if spec is None:
        return s
    t, off = spec
    # any NCL view with unit time stride works (e.g. the channel halves of torch.split, train.py:130)
    assert t.dim() == 3 and t.stride(2) == 1 and t.dtype == torch.float32 and t.is_cuda
    s.p = t.data_ptr()
    s.sb = t.stride(0)
    s.sc = t.stride(1)
    s.C = t.shape[1]
    s.T = t.shape[2]
    s.off = off
    return s


def _dst(spec):
    d = L.MstDst()
    if spec is None:
        return d
    t, off, gate, gscale = spec
    assert t.is_contiguous() and t.dim() == 3
    d.p = t.data_ptr()
    d.sb = t.shape[1] * t.shape[2]
    d.sc = t.shape[2]
    d.C = t.shape[1]
    d.T = t.shape[2]
    d.off = off
    if gate is not None:
        assert gate.shape == t.shape
        d.gate = gate.data_ptr()
        d.gate_scale = gscale
    return d


# Workspace arena: one grow-only scratch buffer per (device, launch stream). Launches on one
# stream are ordered, so consecutive GEMM split-K slabs and loss partials share it instead of
# paying an allocator round trip each. An outgrown buffer is simply dropped: torch's caching
# allocator hands its block out again only in this stream's order, after the launches already
# queued on it. Under stream capture the arena is bypassed (each launch takes a fresh buffer
# from the graph's private pool, torch's capture semantics), so no graph names an arena
# buffer. Requests above ARENA_MAX_BYTES (Griffin-Lim's multi-GB clip chunks) are one-off
# allocations that return to the allocator after the call instead of staying pinned here.
_ARENA = {}
ARENA_MAX_BYTES = 256 << 20


def workspace(nbytes, device):
    """(float32 buffer of >= nbytes, its byte size) for one launch on the current stream."""
    if nbytes == 0:
        return None, 0
    n = (nbytes + 3) // 4
    if torch.cuda.is_current_stream_capturing() or nbytes > ARENA_MAX_BYTES:
        return torch.empty(n, device=device, dtype=torch.float32), 4 * n
    key = (device.index, L.stream().value)
    buf = _ARENA.get(key)
    if buf is None or buf.numel() < n:
        if buf is not None:
            n = min(max(n, 2 * buf.numel()), ARENA_MAX_BYTES // 4)
        _ARENA[key] = None  # release the outgrown block before taking the larger one
        buf = _ARENA[key] = torch.empty(n, device=device, dtype=torch.float32)
    return buf, 4 * buf.numel()


_workspace = workspace


# Optional per-launch GEMM timing (bench.py's roofline leg): when a list is installed, every
# GEMM launch is bracketed by HIP events on torch's current stream (the launch stream).
_GEMM_LOG = None


def gemm_timing(log):
    """Install (list) or remove (None) the GEMM timing log; entries are (start, end, flops, tag)."""
    global _GEMM_LOG
    _GEMM_LOG = log


def _timed(launch, flops, tag, shape=None):
    if _GEMM_LOG is None:
        launch()
        return
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    launch()
    e.record()
    _GEMM_LOG.append((s, e, flops, tag, shape))


def conv_like(*, B, M, Tn, srcs, Tv, taps, a, beta, g, A, A_off=0, sAm, sAc, sAt, dsts, ostride=1,
              ophase=0, alpha=1.0, bias=None, act=L.ACT_NONE, drop_p=0.0, seed=0, splitk=0,
              seed_dev=None):
    lib = _lib()
    d = L.MstConvDesc()
    d.B, d.M, d.Tn, d.taps = B, M, Tn, taps
    d.Ctot = sum(s[0].shape[1] for s in srcs)
    d.a, d.beta, d.g, d.Tv = a, beta, g, Tv
    d.A = A.data_ptr() + 4 * A_off
    d.sAm, d.sAc, d.sAt = sAm, sAc, sAt
    d.src[0] = _src(srcs[0])
    d.src[1] = _src(srcs[1] if len(srcs) > 1 else None)
    d.ostride, d.ophase = ostride, ophase
    d.dst[0] = _dst(dsts[0])
    d.dst[1] = _dst(dsts[1] if len(dsts) > 1 else None)
    d.alpha = alpha
    d.bias = bias.data_ptr() if bias is not None else None
    d.act = act
    d.drop_p = drop_p
    d.seed = seed
    d.seed_dev = seed_dev.data_ptr() if seed_dev is not None else None
    d.splitk = splitk or _FORCE_SPLITK
    ref = ctypes.byref(d)
    need = lib.mst_conv_fwd_workspace_size(ref)  # split-K: splits * M * N * 4 bytes
    ws, nb = _workspace(need, A.device)
    _timed(lambda: L.check(lib.mst_conv_fwd_f32(ref, L.ptr(ws), nb, L.stream()), "mst_conv_fwd_f32"),
           2.0 * M * B * Tn * d.Ctot * taps, "conv", (M, B * Tn, d.Ctot * taps, taps, a, need))


def wgrad_like(*, P, srcs, Tv, taps, a, beta, g, out, ldo, ldc=0, ldt=0, scale=1.0, accumulate=False,
               splitk=0):
    """out[m*ldo + c*ldc + tap*ldt] (+)= scale * sum_{b,t} P[b][m][t] X(b, c, a*t+beta+g*tap);
    ldc = ldt = 0 means the torch layout (ldc = taps, ldt = 1)."""
    lib = _lib()
    d = L.MstWgradDesc()
    B, M, Tk = P.shape
    d.B, d.M, d.Tk, d.taps = B, M, Tk, taps
    d.Ctot = sum(s[0].shape[1] for s in srcs)
    d.a, d.beta, d.g, d.Tv = a, beta, g, Tv
    d.P = P.data_ptr()
    d.sPb = M * Tk
    d.sPc = Tk
    d.src[0] = _src(srcs[0])
    d.src[1] = _src(srcs[1] if len(srcs) > 1 else None)
    d.out = out.data_ptr()
    d.ldo = ldo
    d.ldc, d.ldt = ldc, ldt
    d.scale = scale
    d.accumulate = 1 if accumulate else 0
    d.splitk = splitk or _FORCE_SPLITK
    ref = ctypes.byref(d)
    need = lib.mst_wgrad_workspace_size(ref)  # split-K: splits * M * (source's C * taps) * 4 bytes
    ws, nb = _workspace(need, P.device)
    _timed(lambda: L.check(lib.mst_conv_wgrad_f32(ref, L.ptr(ws), nb, L.stream()),
                           "mst_conv_wgrad_f32"), 2.0 * M * B * Tk * d.Ctot * taps, "wgrad",
           (M, d.Ctot * taps, B * Tk, taps, a, need))


def _wgrad_out(dW):
    """(ldo, ldc, ldt) of a (d0, C, taps) weight-gradient tensor in any layout."""
    return dW.stride(0), dW.stride(1), dW.stride(2)


# ---------------------------------------------------------------- Conv1d k3 p1
# Weights may be in the torch layout or tap-major (model.slot_view): every A operand takes
# its strides from the tensor.
def conv3_fwd(srcs, W, bias, out, act=L.ACT_NONE):
    B, Cout, T = out.shape
    conv_like(B=B, M=Cout, Tn=T, srcs=srcs, Tv=T, taps=3, a=1, beta=-1, g=1, A=W, sAm=W.stride(0),
              sAc=W.stride(1), sAt=W.stride(2), dsts=[(out, 0, None, 1.0)], bias=bias, act=act)


def conv3_dgrad(dY, W, dsts):
    B, Cout, T = dY.shape
    Cin = W.shape[1]
    conv_like(B=B, M=Cin, Tn=T, srcs=[(dY, 0)], Tv=T, taps=3, a=1, beta=1, g=-1, A=W,
              sAm=W.stride(1), sAc=W.stride(0), sAt=W.stride(2), dsts=dsts)


def conv3_wgrad(dY, srcs, dW, accumulate):
    ldo, ldc, ldt = _wgrad_out(dW)
    wgrad_like(P=dY, srcs=srcs, Tv=dY.shape[2], taps=3, a=1, beta=-1, g=1, out=dW, ldo=ldo, ldc=ldc,
               ldt=ldt, accumulate=accumulate)


# ------------------------------------------------- ConvTranspose1d(k, s=2, p=1)
def convT2_out_len(Tin, k):
    return (Tin - 1) * 2 - 2 + k


def convT2_fwd(x, W, bias, out):
    Cin, Cout, k = W.shape
    B, _, Tin = x.shape
    Tout = out.shape[2]
    for p in (0, 1):
        nq = k // 2 if p == 0 else (k + 1) // 2
        Tn = (Tout - p + 1) // 2
        if nq == 0 or Tn <= 0:
            continue
        conv_like(B=B, M=Cout, Tn=Tn, srcs=[(x, 0)], Tv=Tin, taps=nq, a=1, beta=p, g=-1, A=W,
                  A_off=(1 - p) * W.stride(2), sAm=W.stride(1), sAc=W.stride(0), sAt=2 * W.stride(2),
                  dsts=[(out, 0, None, 1.0)], ostride=2, ophase=p, bias=bias)


def convT2_dgrad(dY, W, dsts):
    Cin, Cout, k = W.shape
    B, _, Tout = dY.shape
    Tin = dsts[0][0].shape[2]
    conv_like(B=B, M=Cin, Tn=Tin, srcs=[(dY, 0)], Tv=Tout, taps=k, a=2, beta=-1, g=1, A=W,
              sAm=W.stride(0), sAc=W.stride(1), sAt=W.stride(2), dsts=dsts)


def convT2_wgrad(x, dY, dW, accumulate):
    Cin, Cout, k = dW.shape
    ldo, ldc, ldt = _wgrad_out(dW)
    wgrad_like(P=x, srcs=[(dY, 0)], Tv=dY.shape[2], taps=k, a=2, beta=-1, g=1, out=dW, ldo=ldo,
               ldc=ldc, ldt=ldt, accumulate=accumulate)


# ------------------------------------------- ConvTranspose1d(k=3, s=1, p=1) (lastconv)
def convT1_fwd(x, W, bias, out, alpha=1.0, act=L.ACT_NONE):
    Cin, Cout, k = W.shape
    B, _, T = x.shape
    conv_like(B=B, M=Cout, Tn=T, srcs=[(x, 0)], Tv=T, taps=k, a=1, beta=1, g=-1, A=W,
              sAm=W.stride(1), sAc=W.stride(0), sAt=W.stride(2), dsts=[(out, 0, None, 1.0)],
              alpha=alpha, bias=bias, act=act)


def convT1_dgrad(dY, W, dx, alpha=1.0):
    Cin, Cout, k = W.shape
    B, _, T = dY.shape
    conv_like(B=B, M=Cin, Tn=T, srcs=[(dY, 0)], Tv=T, taps=k, a=1, beta=-1, g=1, A=W,
              sAm=W.stride(0), sAc=W.stride(1), sAt=W.stride(2), dsts=[(dx, 0, None, 1.0)],
              alpha=alpha)


def convT1_wgrad(x, dY, dW, accumulate, scale=1.0):
    ldo, ldc, ldt = _wgrad_out(dW)
    wgrad_like(P=x, srcs=[(dY, 0)], Tv=dY.shape[2], taps=dW.shape[2], a=1, beta=-1, g=1, out=dW,
               ldo=ldo, ldc=ldc, ldt=ldt, scale=scale, accumulate=accumulate)


# ------------------------------------------------------- Linear over NCL channels
def linear_fwd(srcs, W, bias, out, act=L.ACT_NONE, drop_p=0.0, seed=0, seed_dev=None):
    B, Cout, T = out.shape
    Cin = W.shape[1]
    conv_like(B=B, M=Cout, Tn=T, srcs=srcs, Tv=T, taps=1, a=1, beta=0, g=0, A=W, sAm=Cin, sAc=1,
              sAt=1, dsts=[(out, 0, None, 1.0)], bias=bias, act=act, drop_p=drop_p, seed=seed,
              seed_dev=seed_dev)


def linear_dgrad(dY, W, dsts):
    B, Cout, T = dY.shape
    Cin = W.shape[1]
    conv_like(B=B, M=Cin, Tn=T, srcs=[(dY, 0)], Tv=T, taps=1, a=1, beta=0, g=0, A=W, sAm=1,
              sAc=Cin, sAt=1, dsts=dsts)


def linear_wgrad(dY, srcs, dW, accumulate):
    wgrad_like(P=dY, srcs=srcs, Tv=dY.shape[2], taps=1, a=1, beta=0, g=0, out=dW,
               ldo=dW.shape[1], accumulate=accumulate)


# ---------------------------------------------------------- norm / elementwise
def in_lrelu_fwd(y, pool):
    B, C, T = y.shape
    a = torch.empty_like(y)
    pooled = empty(B, C, T // 2, like=y) if pool else None
    mean = empty(B * C, like=y)
    rstd = empty(B * C, like=y)
    L.check(_lib().mst_instnorm_lrelu_fwd_f32(L.ptr(y), B * C, T, IN_EPS, SLOPE, L.ptr(a),
                                              L.ptr(pooled), L.ptr(mean), L.ptr(rstd), L.stream()),
            "instnorm_fwd")
    return a, pooled, mean, rstd


def in_lrelu_bwd(y, mean, rstd, d_a=None, d_pool0=None, d_pool1=None, rowsum=False):
    """IN + LeakyReLU (+ maxpool) backward. rowsum=True also returns the (B, C) per-row sums of
    dy (the producing conv's bias gradient before the batch reduction, bias_grad_rows)."""
    B, C, T = y.shape
    dy = torch.empty_like(y)
    rs = empty(B, C, like=y) if rowsum else None
    L.check(_lib().mst_instnorm_lrelu_bwd_f32(L.ptr(y), L.ptr(mean), L.ptr(rstd), B * C, T, SLOPE,
                                              L.ptr(d_a), L.ptr(d_pool0), L.ptr(d_pool1), L.ptr(dy),
                                              L.ptr(rs), L.stream()), "instnorm_bwd")
    return (dy, rs) if rowsum else dy


def bias_grad_rows(rs, db, accumulate):
    """db (+)= sum over the batch of per-(b, c) row sums (from in_lrelu_bwd(rowsum=True))."""
    B, C = rs.shape
    L.check(_lib().mst_bias_grad_rows_f32(L.ptr(rs), B, C, 1.0, L.ptr(db), 1 if accumulate else 0,
                                          L.stream()), "bias_grad_rows")


def bias_grad(dy, db, accumulate):
    if not dy.is_contiguous() or not db.is_contiguous():
        raise ValueError("bias_grad: contiguous (B, C, T) dy and (C,) db required")
    B, C, T = dy.shape
    L.check(_lib().mst_bias_grad_f32(L.ptr(dy), B, C, T, 1.0, L.ptr(db), 1 if accumulate else 0,
                                     L.stream()), "bias_grad")


def lrelu_bwd(dy, y):
    dx = torch.empty_like(y)
    L.check(_lib().mst_lrelu_bwd_f32(L.ptr(dy), L.ptr(y), y.numel(), SLOPE, L.ptr(dx), L.stream()),
            "lrelu_bwd")
    return dx


def relu_gate_bwd(d, h, scale):
    out = torch.empty_like(h)
    L.check(_lib().mst_relu_gate_bwd_f32(L.ptr(d), L.ptr(h), h.numel(), scale, L.ptr(out),
                                         L.stream()), "relu_gate_bwd")
    return out


def _loss(fn, pred, target):
    lib = _lib()
    n = pred.numel()
    ws, _ = workspace(lib.mst_l1_workspace_size(n) + 8, pred.device)
    loss = torch.empty((), device=pred.device, dtype=torch.float32)
    L.check(getattr(lib, fn)(L.ptr(pred), L.ptr(target), n, L.ptr(loss), L.ptr(ws), L.stream()), fn)
    return loss


def l1_fwd(pred, target):
    return _loss("mst_l1_fwd_f32", pred, target)


def mse_fwd(pred, target):
    return _loss("mst_mse_fwd_f32", pred, target)


def l1_bwd(pred, target, gscale):
    dx = torch.empty_like(pred)
    L.check(_lib().mst_l1_bwd_f32(L.ptr(pred), L.ptr(target), pred.numel(), L.ptr(gscale), L.ptr(dx),
                                  L.stream()), "l1_bwd")
    return dx


def adam(p, g, m, v, lr_step, b1, b2, eps, bc2_sqrt, max_blocks=None):
    """torch.optim.Adam's update (mst_adam_f32). 1 - b1 and 1 - b2 are formed in double here and
    rounded, as torch forms them; max_blocks caps the grid (a background launch)."""
    args = (L.ptr(p), L.ptr(g), L.ptr(m), L.ptr(v), p.numel(), lr_step, b2, 1.0 - b1, 1.0 - b2, eps,
            bc2_sqrt)
    if max_blocks is None:
        L.check(_lib().mst_adam_f32(*args, L.stream()), "adam")
    else:
        L.check(_lib().mst_adam_ex_f32(*args, max_blocks, L.stream()), "adam")


def adam_dev(p, g, m, v, hyper, b1, b2, eps):
    """adam() with (lr_step, bc2_sqrt) read from the 2-float device tensor `hyper`."""
    assert hyper.dtype == torch.float32 and hyper.numel() >= 2 and hyper.is_cuda
    L.check(_lib().mst_adam_dev_f32(L.ptr(p), L.ptr(g), L.ptr(m), L.ptr(v), p.numel(), L.ptr(hyper),
                                    b2, 1.0 - b1, 1.0 - b2, eps, L.stream()), "adam_dev")


def scale_(x, s):
    L.check(_lib().mst_scale_f32(L.ptr(x), x.numel(), s, L.stream()), "scale")


def fill_(x, v):
    L.check(_lib().mst_fill_f32(L.ptr(x), x.numel(), v, L.stream()), "fill")
