"""Device front end: STFT log-power / power / complex, mel spectrogram, iSTFT, Griffin-Lim.

Semantics follow the reference's librosa calls (librosa 0.7-0.9: Hann periodic
window, center=True, reflect padding, n_fft=2048):
  logpow       preprocessing/preprocess.py:47-49   np.log1p(np.abs(librosa.stft(y, 2048, 256))**2)
  melspec      tests/plot_spec.py:20                librosa.feature.melspectrogram (slaney, 128 mels)
  griffinlim   model/inference.py:105-110          librosa.griffinlim(n_iter, momentum=0.99)
All compute runs in libmst_hip's FFT kernels (fft.hip) behind the torch.ops.mst.* custom ops
(ops.py); inputs/outputs are CUDA tensors.
"""
import math

import numpy as np
import torch

from . import _lib as L
from . import ops as _ops  # noqa: F401  (registers torch.ops.mst.*)

N_FFT = 2048


def _as_batch(x):
    if x.dim() == 1:
        return x.unsqueeze(0), True
    return x, False


def _check_signal(x):
    if not x.is_cuda:
        raise RuntimeError("spectral kernels need a CUDA tensor")
    return x.contiguous().float()


def n_frames(L_samples, hop):
    return 1 + L_samples // hop


def stft_logpow(x, hop=256, n_fft=N_FFT, pad_mode="reflect"):
    """(L,) or (B, L) signal -> (F, T) / (B, F, T) log1p(|STFT|^2) (torch.ops.mst.stft_logpow)."""
    x, single = _as_batch(_check_signal(x))
    out = torch.ops.mst.stft_logpow(x, n_fft, hop, _pad_code(pad_mode))
    return out[0] if single else out


def stft_power(x, hop=256, n_fft=N_FFT, pad_mode="reflect"):
    """|STFT|^2, same layout as stft_logpow (torch.ops.mst.stft_power)."""
    x, single = _as_batch(_check_signal(x))
    out = torch.ops.mst.stft_power(x, n_fft, hop, _pad_code(pad_mode))
    return out[0] if single else out


def _pad_code(pad_mode):
    return {"reflect": L.PAD_REFLECT, "constant": L.PAD_CONSTANT}[pad_mode]


def stft_complex(x, hop=256, n_fft=N_FFT, pad_mode="reflect"):
    """Complex STFT, frame-major: (B, T, F) complex64 view of a (B, T, F, 2) buffer."""
    x, single = _as_batch(_check_signal(x))
    out = torch.view_as_complex(torch.ops.mst.stft_complex(x, n_fft, hop, _pad_code(pad_mode)))
    return out[0] if single else out


def istft(X, hop=256):
    """Inverse of stft_complex: (B, T, F) complex (frame-major) -> (B, hop*(T-1))."""
    single = X.dim() == 2
    if single:
        X = X.unsqueeze(0)
    y = torch.ops.mst.istft(torch.view_as_real(X.contiguous()).contiguous(), int(hop))
    return y[0] if single else y


# ------------------------------------------------- differentiable iSTFT (training losses)
_WSS_CACHE = {}


def _inv_wss(T, hop, n_fft, device):
    """1 / window-sum-square at the kept (center-trimmed) samples, 0 where it vanishes."""
    key = (T, hop, n_fft, str(device))
    if key not in _WSS_CACHE:
        n = torch.arange(n_fft, dtype=torch.float64)
        w2 = (0.5 - 0.5 * torch.cos(2 * math.pi * n / n_fft)) ** 2
        wss = torch.zeros(n_fft + hop * (T - 1), dtype=torch.float64)
        for k in range(T):
            wss[k * hop:k * hop + n_fft] += w2
        wss = wss[n_fft // 2:n_fft // 2 + hop * (T - 1)]
        tiny = torch.finfo(torch.float32).tiny
        inv = torch.where(wss > tiny, 1.0 / wss.clamp_min(tiny), torch.zeros_like(wss))
        _WSS_CACHE[key] = inv.float().to(device)
    return _WSS_CACHE[key]


def istft_autograd(X, hop=256):
    """Differentiable istft: (B, T, F) complex frame-major -> (B, hop*(T-1))."""
    single = X.dim() == 2
    Xb = (X.unsqueeze(0) if single else X).contiguous()
    if not Xb.is_cuda:
        raise RuntimeError("istft_autograd needs a CUDA tensor")
    # mst::istft's registered backward is the adjoint (a constant-padded STFT of g / wss)
    y = torch.ops.mst.istft(torch.view_as_real(Xb), int(hop))
    return y[0] if single else y


def render_logpow(S, P):
    """(B, F, T) log-power -> (B, T, F, 2) complex spectrum sqrt(expm1(clip(S, 0, 20))) * P/|P|
    (inference.py:109's inversion, with the phase of the held spectrum P: (B, T, F, 2) float or
    (B, T, F) complex). One fused transpose kernel each way (render.hip); differentiable in S."""
    if torch.is_complex(P):
        P = torch.view_as_real(P)
    return torch.ops.mst.render_logpow(S, P.detach().contiguous())


MSS_PHASES = ("target", "griffinlim")


def spectrogram_mss_loss(S_pred, target_audio=None, phase="target", hop=256, alpha=1.0, eps=1e-7,
                         sizes=None, S_target=None, gl_iters=8):
    """The README's intended loss (README.md:23; the reference's engel_loss stub,
    train.py:119-123) as a training loss on the model's log-power output: render audio
    y = istft(sqrt(expm1(clip(S_pred, 0, 20))) * phase) and take the multi-scale spectral loss
    against the target waveform; gradients flow to S_pred through the iSTFT adjoint with the phase
    held constant.

    phase: "target"      the STFT phase of target_audio;
           "griffinlim"  the phase of S_pred's own Griffin-Lim reconstruction (gl_iters iterations
                         from all-ones phases, no gradient): the audio inference would synthesise
                         (inference.py:105-110), rendered from the model's magnitude;
           a tensor      any held (B, T, F, 2) / complex (B, T, F) spectrum.
    target_audio: (B, hop (T - 1)) waveform, or None with S_target (B, F, T) log-power: the target
    is then S_target's Griffin-Lim reconstruction (the reference's HDF5 data holds spectrograms
    only, io_manager.py:64-76). Built-defined loss: parity unpinned against the reference."""
    B, F, T = S_pred.shape
    n_fft = 2 * (F - 1)
    with torch.no_grad():
        if target_audio is None:
            if S_target is None:
                raise ValueError("spectrogram_mss_loss needs target_audio or S_target")
            target_audio = griffinlim(S_target, n_iter=gl_iters, hop_length=hop, init=None,
                                      from_logpow=True)
        if target_audio.shape != (B, hop * (T - 1)):
            raise ValueError("target_audio must be (B, hop*(T-1))")
        if isinstance(phase, torch.Tensor):
            P = phase
        elif phase == "target":
            P = stft_complex(target_audio.contiguous(), hop=hop, n_fft=n_fft)
        elif phase == "griffinlim":
            y_gl = griffinlim(S_pred.detach(), n_iter=gl_iters, hop_length=hop, init=None,
                              from_logpow=True)
            P = stft_complex(y_gl, hop=hop, n_fft=n_fft)
        else:
            raise ValueError(f"phase={phase!r}: one of {MSS_PHASES} or a tensor")
    X = render_logpow(S_pred, P)
    y = torch.ops.mst.istft(X, int(hop))
    return multiscale_spectral_loss(y, target_audio.detach(), alpha=alpha, eps=eps,
                                    sizes=MSS_SIZES if sizes is None else sizes)


# ------------------------------------------------------------------- mel
def _hz_to_mel(f):
    f = np.asarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    lin = f / f_sp
    log_t = 1000.0 / f_sp + np.log(np.maximum(f, 1e-300) / 1000.0) / (np.log(6.4) / 27.0)
    return np.where(f >= 1000.0, log_t, lin)


def _mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    min_log_mel = 1000.0 / f_sp
    return np.where(m >= min_log_mel, 1000.0 * np.exp(np.log(6.4) / 27.0 * (m - min_log_mel)), f_sp * m)


def mel_basis(sr, n_fft=N_FFT, n_mels=128, fmin=0.0, fmax=None):
    """Slaney-normalised mel filterbank (librosa.filters.mel defaults) as float32 (n_mels, F)."""
    fmax = sr / 2.0 if fmax is None else fmax
    nb = 1 + n_fft // 2
    fftfreqs = np.linspace(0, sr / 2.0, nb)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fftfreqs[None, :]
    lower = -ramps[:-2] / fdiff[:-1, None]
    upper = ramps[2:] / fdiff[1:, None]
    w = np.maximum(0, np.minimum(lower, upper))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return w.astype(np.float32)


_MEL_CACHE = {}


def _mel_tables(sr, n_fft, n_mels, device):
    key = (sr, n_fft, n_mels, str(device))
    if key not in _MEL_CACHE:
        w = mel_basis(sr, n_fft, n_mels)
        start, length, woff, vals = [], [], [], []
        off = 0
        for m in range(n_mels):
            nz = np.nonzero(w[m])[0]
            s, e = (int(nz[0]), int(nz[-1]) + 1) if nz.size else (0, 0)
            start.append(s)
            length.append(e - s)
            woff.append(off)
            vals.append(w[m, s:e])
            off += e - s
        vals = np.concatenate(vals) if off else np.zeros(1, np.float32)
        mk = lambda a, dt: torch.tensor(np.asarray(a), dtype=dt, device=device)  # noqa: E731
        _MEL_CACHE[key] = (mk(start, torch.int32), mk(length, torch.int32), mk(woff, torch.int32),
                           mk(vals, torch.float32))
    return _MEL_CACHE[key]


def melspectrogram(x, sr, n_fft=N_FFT, hop_length=256, n_mels=128, pad_mode="reflect"):
    """librosa.feature.melspectrogram(y, sr, n_fft, hop_length) (power 2, slaney, 128 mels)."""
    x, single = _as_batch(_check_signal(x))
    st, ln, wo, w = _mel_tables(sr, n_fft, n_mels, x.device)
    out = torch.ops.mst.melspectrogram(x, n_fft, hop_length, _pad_code(pad_mode), st, ln, wo, w)
    return out[0] if single else out


# ------------------------------------------------------------ Griffin-Lim
def random_angles(shape_btf, seed, device):
    """Unit phases exp(2 pi i U[0,1)) like librosa's init='random' (seeded), frame-major."""
    rng = np.random.RandomState(seed)
    ang = np.exp(2j * np.pi * rng.rand(*shape_btf)).astype(np.complex64)
    return torch.view_as_real(torch.from_numpy(ang)).contiguous().to(device)


def griffinlim(S, n_iter=60, hop_length=256, momentum=0.99, init="random", seed=0,
               from_logpow=False):
    """librosa.griffinlim on the device. S: (F, T) or (B, F, T) magnitudes (or log-power when
    from_logpow, inverted as sqrt(expm1(clip(S, 0, 20))) like inference.py:109).
    init: 'random' (seeded), None/'ones', or a (B, T, F, 2) float tensor of unit phases."""
    S, single = (S.unsqueeze(0), True) if S.dim() == 2 else (S, False)
    S = S.contiguous().float()
    if not S.is_cuda:
        raise RuntimeError("griffinlim needs a CUDA tensor")
    B, F, T = S.shape
    if momentum < 0:
        raise ValueError("griffinlim() called with momentum < 0")
    if isinstance(init, torch.Tensor):
        ang = init.contiguous().float()
    elif init == "random":
        ang = random_angles((B, T, F), seed, S.device)
    elif init is None or init == "ones":
        ang = None
    else:
        raise ValueError(f"init={init!r} must be 'random', None or a tensor")
    y = torch.ops.mst.griffinlim(S, int(n_iter), int(hop_length), float(momentum), ang,
                                 bool(from_logpow))
    return y[0] if single else y


# ------------------------------------------------------- multi-scale spectral loss
MSS_SIZES = (2048, 1024, 512, 256, 128, 64)


def multiscale_spectral_loss(pred, target, alpha=1.0, eps=1e-7, sizes=MSS_SIZES):
    """DDSP multi-scale spectral loss (README.md:23; the reference's `engel_loss` stub,
    train.py:119-123 — this build owns the definition, parity unpinned):

      sum_n mean|S_n(pred) - S_n(target)| + alpha * mean|log(S_n(pred)+eps) - log(S_n(target)+eps)|

    S_n = |STFT| with n_fft = n, hop n/4, periodic Hann, center + reflect pad; means over every
    (clip, bin, frame). pred/target: (L,) or (B, L) CUDA waveforms. Differentiable in pred."""
    if pred.shape != target.shape:
        raise ValueError("pred and target must have the same shape")
    pred_b, _ = _as_batch(_check_signal(pred))
    tgt_b, _ = _as_batch(_check_signal(target).detach())
    want = torch.is_grad_enabled() and pred_b.requires_grad
    loss, _ = torch.ops.mst.mss_loss(pred_b, tgt_b, [int(n) for n in sizes], float(alpha),
                                     float(eps), want)
    return loss


def spectral_convergence(S, y, hop=256):
    """|| |STFT(y)| - S ||_F / ||S||_F for (B, F, T) magnitudes (diagnostic)."""
    P = stft_power(y, hop).clamp_min(0).sqrt()
    return (torch.linalg.vector_norm(P - S) / torch.linalg.vector_norm(S)).item()


__all__ = ["stft_logpow", "stft_power", "stft_complex", "istft", "melspectrogram", "mel_basis",
           "griffinlim", "random_angles", "spectral_convergence", "n_frames",
           "multiscale_spectral_loss", "MSS_SIZES", "math", "istft_autograd",
           "spectrogram_mss_loss", "render_logpow", "MSS_PHASES"]
