"""torch.library custom ops over libmst_hip (namespace `mst`): `torch.ops.mst.*`.

Each op has a fake (meta) kernel, so FakeTensorMode, torch.compile / torch.export tracing and
shape propagation see the op without running it; the differentiable ones register their
backward with `register_autograd`. The CUDA implementations are the same C-ABI launches the
Python drop-ins use (include/mst.h); there is no CPU implementation (a CPU tensor raises).

  op                                 reference (file:line)
  stft_logpow / stft_power           preprocessing/preprocess.py:47-49
  stft_complex (frame-major)         librosa.stft behind model/inference.py:105-110
  istft (differentiable)             librosa.istft behind the same Griffin-Lim (+ istft_backward)
  render_logpow (differentiable)     model/inference.py:109 (magnitude inversion) with a held phase
  melspectrogram                     tests/plot_spec.py:20
  griffinlim                         model/inference.py:105-110, tests/test_griffinlim.py:23
  mss_loss (differentiable)          README.md:23, model/train.py:119-123 (engel_loss stub)
  l1_loss (differentiable)           model/train.py:132-135,140 (nn.L1Loss)
  mse_loss                           model/train.py:158 (nn.MSELoss, test())
  onoff                              preprocessing/preprocess.py:148-155
  conv1d_k3 (differentiable)         model/model.py:14-22 (nn.Conv1d(k=3, padding=1))
  conv_transpose1d (differentiable)  model/model.py:24-31,242 (nn.ConvTranspose1d, s=2 p=1 / s=1 p=1)
  linear_ncl (differentiable)        model/model.py:98-99,104-107 (nn.Linear over NCL channels)

pad_mode ints: 0 reflect, 1 constant (MST_PAD_*).
"""
import ctypes
from typing import List, Optional, Tuple

import torch
from torch import Tensor
from torch.library import custom_op

from . import _lib as L
from . import kernels as K

N_FFT = 2048


def _signal(x):
    if not x.is_cuda:
        raise RuntimeError("torch.ops.mst: CUDA (HIP) tensors only; there is no CPU path")
    return x.contiguous().float()


def _frames(n, hop):
    return 1 + n // hop


# ------------------------------------------------------------------ STFT family
def _stft_real(fn, x, n_fft, hop, pad_mode):
    x = _signal(x)
    B, Ls = x.shape
    out = torch.empty(B, n_fft // 2 + 1, _frames(Ls, hop), device=x.device, dtype=torch.float32)
    L.check(getattr(L.load(), fn)(L.ptr(x), B, Ls, n_fft, hop, pad_mode, L.ptr(out), L.stream()), fn)
    return out


@custom_op("mst::stft_logpow", mutates_args=())
def stft_logpow(x: Tensor, n_fft: int, hop: int, pad_mode: int) -> Tensor:
    """(B, L) -> (B, n_fft/2 + 1, 1 + L/hop) log1p(|STFT|^2)."""
    return _stft_real("mst_stft_logpow_f32", x, n_fft, hop, pad_mode)


@custom_op("mst::stft_power", mutates_args=())
def stft_power(x: Tensor, n_fft: int, hop: int, pad_mode: int) -> Tensor:
    """(B, L) -> (B, F, T) |STFT|^2."""
    return _stft_real("mst_stft_power_f32", x, n_fft, hop, pad_mode)


@stft_logpow.register_fake
@stft_power.register_fake
def _stft_real_fake(x, n_fft, hop, pad_mode):
    B, Ls = x.shape
    return x.new_empty(B, n_fft // 2 + 1, _frames(Ls, hop), dtype=torch.float32)


@custom_op("mst::stft_complex", mutates_args=())
def stft_complex(x: Tensor, n_fft: int, hop: int, pad_mode: int) -> Tensor:
    """(B, L) -> (B, T, F, 2) frame-major complex STFT (real/imag interleaved)."""
    x = _signal(x)
    B, Ls = x.shape
    out = torch.empty(B, _frames(Ls, hop), n_fft // 2 + 1, 2, device=x.device, dtype=torch.float32)
    L.check(L.load().mst_stft_complex_f32(L.ptr(x), B, Ls, n_fft, hop, pad_mode, L.ptr(out),
                                          L.stream()), "stft_complex")
    return out


@stft_complex.register_fake
def _stft_complex_fake(x, n_fft, hop, pad_mode):
    B, Ls = x.shape
    return x.new_empty(B, _frames(Ls, hop), n_fft // 2 + 1, 2, dtype=torch.float32)


@custom_op("mst::istft", mutates_args=())
def istft(X: Tensor, hop: int) -> Tensor:
    """(B, T, F, 2) frame-major complex -> (B, hop (T - 1)) (librosa.istft, center, Hann)."""
    X = _signal(X)
    B, T, F, _ = X.shape
    y = torch.empty(B, hop * (T - 1), device=X.device, dtype=torch.float32)
    L.check(L.load().mst_istft_f32(L.ptr(X), B, F, T, hop, L.ptr(y), L.stream()), "istft")
    return y


@istft.register_fake
def _istft_fake(X, hop):
    B, T, F, _ = X.shape
    return X.new_empty(B, hop * (T - 1), dtype=torch.float32)


def _istft_setup(ctx, inputs, output):
    X, hop = inputs
    ctx.hop, ctx.T, ctx.F = hop, X.shape[1], X.shape[2]


@custom_op("mst::istft_backward", mutates_args=())
def istft_backward(grad: Tensor, n_frames: int, n_bins: int, hop: int) -> Tensor:
    """Adjoint of mst::istft. y = istft(X) is linear; with h = g / wss on the kept samples
    (zeros in the trimmed margins, i.e. center padding with constants),
    dL/dX[k, f] = (c_f / n_fft) * rfft(w * h[k*hop : k*hop + n_fft])[f], c_f = 1 at f = 0 and
    n_fft/2, else 2 (irfft's Hermitian weights): a constant-padded stft_complex of h."""
    from .spectral import _inv_wss
    g = _signal(grad)
    n_fft = 2 * (n_bins - 1)
    h = (g * _inv_wss(n_frames, hop, n_fft, g.device)).contiguous()
    G = stft_complex(h, n_fft, hop, L.PAD_CONSTANT)
    c = torch.full((n_bins, 1), 2.0 / n_fft, device=g.device)
    c[0] = c[-1] = 1.0 / n_fft
    return G * c


@istft_backward.register_fake
def _istft_backward_fake(grad, n_frames, n_bins, hop):
    return grad.new_empty(grad.shape[0], n_frames, n_bins, 2, dtype=torch.float32)


def _istft_backward(ctx, g):
    return torch.ops.mst.istft_backward(g, ctx.T, ctx.F, ctx.hop), None


istft.register_autograd(_istft_backward, setup_context=_istft_setup)


@custom_op("mst::render_logpow", mutates_args=())
def render_logpow(S: Tensor, P: Tensor) -> Tensor:
    """(B, F, T) log-power, (B, T, F, 2) held complex spectrum -> (B, T, F, 2)
    sqrt(expm1(clip(S, 0, 20))) * P / |P| (inference.py:109's inversion with P's phase)."""
    S, P = _signal(S), _signal(P)
    B, F, T = S.shape
    if tuple(P.shape) != (B, T, F, 2):
        raise ValueError("render_logpow: P must be (B, T, F, 2)")
    X = torch.empty(B, T, F, 2, device=S.device, dtype=torch.float32)
    L.check(L.load().mst_render_logpow_f32(L.ptr(S), L.ptr(P), B, F, T, L.ptr(X), L.stream()),
            "render_logpow")
    return X


@render_logpow.register_fake
def _render_fake(S, P):
    B, F, T = S.shape
    return S.new_empty(B, T, F, 2, dtype=torch.float32)


@custom_op("mst::render_logpow_backward", mutates_args=())
def render_logpow_backward(S: Tensor, P: Tensor, grad: Tensor) -> Tensor:
    """d/dS of render_logpow with P held: Re(conj(P/|P|) grad) * e^S / (2 M) inside (0, 20)."""
    S, P, g = _signal(S), _signal(P), _signal(grad)
    B, F, T = S.shape
    dS = torch.empty_like(S)
    L.check(L.load().mst_render_logpow_bwd_f32(L.ptr(S), L.ptr(P), L.ptr(g), B, F, T, L.ptr(dS),
                                               L.stream()), "render_logpow_backward")
    return dS


@render_logpow_backward.register_fake
def _render_backward_fake(S, P, grad):
    return torch.empty_like(S)


def _render_setup(ctx, inputs, output):
    S, P = inputs
    ctx.save_for_backward(S, P)


def _render_backward(ctx, g):
    S, P = ctx.saved_tensors
    return torch.ops.mst.render_logpow_backward(S, P, g), None


render_logpow.register_autograd(_render_backward, setup_context=_render_setup)


@custom_op("mst::melspectrogram", mutates_args=())
def melspectrogram(x: Tensor, n_fft: int, hop: int, pad_mode: int, start: Tensor, length: Tensor,
                   woff: Tensor, weights: Tensor) -> Tensor:
    """(B, L) -> (B, n_mels, T) mel power spectrogram; the filterbank is sparse per band
    (spectral._mel_tables)."""
    x = _signal(x)
    B, Ls = x.shape
    n_mels = start.shape[0]
    out = torch.empty(B, n_mels, _frames(Ls, hop), device=x.device, dtype=torch.float32)
    L.check(L.load().mst_stft_mel_f32(L.ptr(x), B, Ls, n_fft, hop, pad_mode, L.ptr(start),
                                      L.ptr(length), L.ptr(woff), L.ptr(weights), n_mels,
                                      L.ptr(out), L.stream()), "stft_mel")
    return out


@melspectrogram.register_fake
def _mel_fake(x, n_fft, hop, pad_mode, start, length, woff, weights):
    B, Ls = x.shape
    return x.new_empty(B, start.shape[0], _frames(Ls, hop), dtype=torch.float32)


@custom_op("mst::griffinlim", mutates_args=())
def griffinlim(S: Tensor, n_iter: int, hop: int, momentum: float, angles: Optional[Tensor],
               mag_from_logpow: bool) -> Tensor:
    """(B, F, T) magnitudes (or log-power) -> (B, hop (T - 1)) signal; angles (B, T, F, 2) or
    None (all ones)."""
    S = _signal(S)
    B, F, T = S.shape
    lib = L.load()
    ws, ws_bytes = K.workspace(lib.mst_griffinlim_workspace_size(B, F, T, hop) + 256, S.device)
    y = torch.empty(B, hop * (T - 1), device=S.device, dtype=torch.float32)
    ang = angles.contiguous().float() if angles is not None else None
    L.check(lib.mst_griffinlim_f32(L.ptr(S), B, F, T, hop, n_iter, float(momentum), L.ptr(ang),
                                   1 if mag_from_logpow else 0, L.ptr(y), L.ptr(ws),
                                   ws_bytes, L.stream()), "griffinlim")
    return y


@griffinlim.register_fake
def _griffinlim_fake(S, n_iter, hop, momentum, angles, mag_from_logpow):
    B, F, T = S.shape
    return S.new_empty(B, hop * (T - 1), dtype=torch.float32)


# --------------------------------------------------------------- losses
@custom_op("mst::mss_loss", mutates_args=())
def mss_loss(pred: Tensor, target: Tensor, sizes: List[int], alpha: float, eps: float,
             with_grad: bool) -> Tuple[Tensor, Tensor]:
    """Multi-scale spectral loss (scalar) and d loss / d pred ((B, L); zeros-size when
    with_grad is False), one pass over the frames (mss.hip)."""
    pred, target = _signal(pred), _signal(target)
    lib = L.load()
    B, Ls = pred.shape
    arr = (ctypes.c_int32 * len(sizes))(*sizes)
    nbytes = lib.mst_mss_workspace_size(B, Ls, len(sizes), arr)
    if nbytes == 0:
        raise ValueError(f"mss_loss: bad sizes {sizes} for length {Ls} (powers of two in "
                         "[64, 2048], at most 8, signal longer than n/2)")
    ws, ws_bytes = K.workspace(nbytes + 64, pred.device)
    loss = torch.empty((), device=pred.device, dtype=torch.float32)
    d = torch.empty_like(pred) if with_grad else pred.new_empty(0)
    L.check(lib.mst_mss_loss_f32(L.ptr(pred), L.ptr(target), B, Ls, len(sizes), arr, float(alpha),
                                 float(eps), L.ptr(loss), L.ptr(d) if with_grad else None, L.ptr(ws),
                                 ws_bytes, L.stream()), "mss_loss")
    return loss, d


@mss_loss.register_fake
def _mss_fake(pred, target, sizes, alpha, eps, with_grad):
    return pred.new_empty((), dtype=torch.float32), (pred.new_empty(pred.shape) if with_grad
                                                     else pred.new_empty(0))


def _mss_setup(ctx, inputs, output):
    ctx.save_for_backward(output[1])


def _mss_backward(ctx, g_loss, g_d):
    (d,) = ctx.saved_tensors
    if d.numel() == 0:
        if ctx.needs_input_grad[0]:
            raise RuntimeError("mst::mss_loss was called with with_grad=False on a pred that "
                               "requires grad: call it with with_grad=True (or use "
                               "spectral.multiscale_spectral_loss, which chooses the flag)")
        return None, None, None, None, None, None
    return d * g_loss, None, None, None, None, None


mss_loss.register_autograd(_mss_backward, setup_context=_mss_setup)


@custom_op("mst::l1_loss", mutates_args=())
def l1_loss(pred: Tensor, target: Tensor) -> Tensor:
    """nn.L1Loss(): mean |pred - target| (double-precision partial sums, deterministic)."""
    return K.l1_fwd(_signal(pred), _signal(target))


@custom_op("mst::l1_loss_backward", mutates_args=())
def l1_loss_backward(pred: Tensor, target: Tensor, grad: Tensor) -> Tensor:
    """grad * sign(pred - target) / numel (sign(0) = 0)."""
    return K.l1_bwd(_signal(pred), _signal(target), grad.contiguous().float())


@l1_loss.register_fake
def _l1_fake(pred, target):
    return pred.new_empty((), dtype=torch.float32)


@l1_loss_backward.register_fake
def _l1_bwd_fake(pred, target, grad):
    return pred.new_empty(pred.shape, dtype=torch.float32)


def _l1_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs)


def _l1_backward(ctx, g):
    pred, target = ctx.saved_tensors
    return torch.ops.mst.l1_loss_backward(pred, target, g), None


l1_loss.register_autograd(_l1_backward, setup_context=_l1_setup)


@custom_op("mst::mse_loss", mutates_args=())
def mse_loss(pred: Tensor, target: Tensor) -> Tensor:
    """nn.MSELoss() forward (evaluation, train.py:158)."""
    return K.mse_fwd(_signal(pred), _signal(target))


@mse_loss.register_fake
def _mse_fake(pred, target):
    return pred.new_empty((), dtype=torch.float32)


@custom_op("mst::onoff", mutates_args=())
def onoff(roll: Tensor) -> Tuple[Tensor, Tensor]:
    """(B, T, 128) velocities -> binarised roll and onset/offset (+1 / -1), both (B, T, 128)."""
    roll = _signal(roll)
    B, T, _ = roll.shape
    b, o = torch.empty_like(roll), torch.empty_like(roll)
    L.check(L.load().mst_onoff_f32(L.ptr(roll), B, T, L.ptr(b), L.ptr(o), L.stream()), "onoff")
    return b, o


@onoff.register_fake
def _onoff_fake(roll):
    return roll.new_empty(roll.shape), roll.new_empty(roll.shape)


# --------------------------------------------------------------- layers (NCL)
def _bias_out(b, ref):
    return b.contiguous().float() if b is not None else None


@custom_op("mst::conv1d_k3", mutates_args=())
def conv1d_k3(x: Tensor, weight: Tensor, bias: Optional[Tensor]) -> Tensor:
    """nn.Conv1d(Cin, Cout, 3, padding=1): (B, Cin, T) -> (B, Cout, T)."""
    x = _signal(x)
    B, _, T = x.shape
    y = torch.empty(B, weight.shape[0], T, device=x.device, dtype=torch.float32)
    K.conv3_fwd([(x, 0)], weight.float(), _bias_out(bias, y), y)
    return y


@conv1d_k3.register_fake
def _conv1d_k3_fake(x, weight, bias):
    return x.new_empty(x.shape[0], weight.shape[0], x.shape[2], dtype=torch.float32)


@custom_op("mst::conv1d_k3_backward", mutates_args=())
def conv1d_k3_backward(grad: Tensor, x: Tensor, weight: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    """(d x, d weight, d bias) of conv1d_k3."""
    g, x = _signal(grad), _signal(x)
    dx = torch.empty_like(x)
    K.conv3_dgrad(g, weight.float(), [(dx, 0, None, 1.0)])
    dW = torch.empty(weight.shape, device=x.device, dtype=torch.float32)
    K.conv3_wgrad(g, [(x, 0)], dW, False)
    db = torch.empty(weight.shape[0], device=x.device, dtype=torch.float32)
    K.bias_grad(g, db, False)
    return dx, dW, db


@conv1d_k3_backward.register_fake
def _conv1d_k3_bwd_fake(grad, x, weight):
    return (x.new_empty(x.shape), weight.new_empty(weight.shape, dtype=torch.float32),
            weight.new_empty(weight.shape[0], dtype=torch.float32))


def _conv_setup(ctx, inputs, output):
    x, w, b = inputs
    ctx.save_for_backward(x, w)
    ctx.has_bias = b is not None


def _conv1d_k3_backward(ctx, g):
    x, w = ctx.saved_tensors
    dx, dW, db = torch.ops.mst.conv1d_k3_backward(g, x, w)
    return dx, dW, (db if ctx.has_bias else None)


conv1d_k3.register_autograd(_conv1d_k3_backward, setup_context=_conv_setup)


@custom_op("mst::conv_transpose1d", mutates_args=())
def conv_transpose1d(x: Tensor, weight: Tensor, bias: Optional[Tensor], stride: int) -> Tensor:
    """nn.ConvTranspose1d(Cin, Cout, k, stride, padding=1) for stride 2 (UpConv, k in
    {2, 3, 4, 6}: the reference's up-kernels) or stride 1 (k = 3, lastconv):
    (B, Cin, T) -> (B, Cout, Tout)."""
    _convT_check(weight.shape[2], stride)
    x = _signal(x)
    B, _, Tin = x.shape
    k = weight.shape[2]
    w = weight.float()
    if stride == 2:
        y = torch.empty(B, weight.shape[1], K.convT2_out_len(Tin, k), device=x.device,
                        dtype=torch.float32)
        K.convT2_fwd(x, w, _bias_out(bias, y), y)
    else:
        y = torch.empty(B, weight.shape[1], Tin, device=x.device, dtype=torch.float32)
        K.convT1_fwd(x, w, _bias_out(bias, y), y)
    return y


def _convT_check(k, stride):
    if not ((stride == 2 and k in (2, 3, 4, 6)) or (stride == 1 and k == 3)):
        raise ValueError("mst::conv_transpose1d: stride 2 with k in {2, 3, 4, 6} or stride 1 "
                         f"with k = 3 (got stride {stride}, k {k})")


@conv_transpose1d.register_fake
def _convT_fake(x, weight, bias, stride):
    Tin, k = x.shape[2], weight.shape[2]
    _convT_check(k, stride)
    Tout = (Tin - 1) * 2 - 2 + k if stride == 2 else Tin
    return x.new_empty(x.shape[0], weight.shape[1], Tout, dtype=torch.float32)


@custom_op("mst::conv_transpose1d_backward", mutates_args=())
def conv_transpose1d_backward(grad: Tensor, x: Tensor, weight: Tensor,
                              stride: int) -> Tuple[Tensor, Tensor, Tensor]:
    g, x = _signal(grad), _signal(x)
    w = weight.float()
    dx = torch.empty_like(x)
    dW = torch.empty(weight.shape, device=x.device, dtype=torch.float32)
    if stride == 2:
        K.convT2_dgrad(g, w, [(dx, 0, None, 1.0)])
        K.convT2_wgrad(x, g, dW, False)
    else:
        K.convT1_dgrad(g, w, dx)
        K.convT1_wgrad(x, g, dW, False)
    db = torch.empty(weight.shape[1], device=x.device, dtype=torch.float32)
    K.bias_grad(g, db, False)
    return dx, dW, db


@conv_transpose1d_backward.register_fake
def _convT_bwd_fake(grad, x, weight, stride):
    return (x.new_empty(x.shape), weight.new_empty(weight.shape, dtype=torch.float32),
            weight.new_empty(weight.shape[1], dtype=torch.float32))


def _convT_setup(ctx, inputs, output):
    x, w, b, stride = inputs
    ctx.save_for_backward(x, w)
    ctx.has_bias, ctx.stride = b is not None, stride


def _convT_backward(ctx, g):
    x, w = ctx.saved_tensors
    dx, dW, db = torch.ops.mst.conv_transpose1d_backward(g, x, w, ctx.stride)
    return dx, dW, (db if ctx.has_bias else None), None


conv_transpose1d.register_autograd(_convT_backward, setup_context=_convT_setup)


@custom_op("mst::linear_ncl", mutates_args=())
def linear_ncl(x: Tensor, weight: Tensor, bias: Optional[Tensor]) -> Tensor:
    """nn.Linear applied over the channels of an NCL tensor (DenseConcat's transpose ->
    Linear -> transpose, model.py:104-107 without the transposes): (B, Cin, T) -> (B, Cout, T)."""
    x = _signal(x)
    B, _, T = x.shape
    y = torch.empty(B, weight.shape[0], T, device=x.device, dtype=torch.float32)
    K.linear_fwd([(x, 0)], weight.contiguous().float(), _bias_out(bias, y), y)
    return y


@linear_ncl.register_fake
def _linear_fake(x, weight, bias):
    return x.new_empty(x.shape[0], weight.shape[0], x.shape[2], dtype=torch.float32)


@custom_op("mst::linear_ncl_backward", mutates_args=())
def linear_ncl_backward(grad: Tensor, x: Tensor, weight: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    g, x = _signal(grad), _signal(x)
    w = weight.contiguous().float()
    dx = torch.empty_like(x)
    K.linear_dgrad(g, w, [(dx, 0, None, 1.0)])
    dW = torch.empty(weight.shape, device=x.device, dtype=torch.float32)
    K.linear_wgrad(g, [(x, 0)], dW, False)
    db = torch.empty(weight.shape[0], device=x.device, dtype=torch.float32)
    K.bias_grad(g, db, False)
    return dx, dW, db


@linear_ncl_backward.register_fake
def _linear_bwd_fake(grad, x, weight):
    return (x.new_empty(x.shape), weight.new_empty(weight.shape, dtype=torch.float32),
            weight.new_empty(weight.shape[0], dtype=torch.float32))


def _linear_backward(ctx, g):
    x, w = ctx.saved_tensors
    dx, dW, db = torch.ops.mst.linear_ncl_backward(g, x, w)
    return dx, dW, (db if ctx.has_bias else None)


linear_ncl.register_autograd(_linear_backward, setup_context=_conv_setup)

OPS = ("stft_logpow", "stft_power", "stft_complex", "istft", "istft_backward", "render_logpow",
       "render_logpow_backward", "melspectrogram",
       "griffinlim", "mss_loss", "l1_loss", "l1_loss_backward", "mse_loss", "onoff", "conv1d_k3",
       "conv1d_k3_backward", "conv_transpose1d", "conv_transpose1d_backward", "linear_ncl",
       "linear_ncl_backward")
