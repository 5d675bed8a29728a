"""float64 NumPy restatement of the librosa calls on the hot path — parity oracle.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

librosa is absent from every interpreter in the build container and version-
unpinned by the reference (no requirements file), so this restates its
published algorithm (librosa 0.7-0.9 era: center=True, pad_mode='reflect',
float64 window and FFT, complex64 storage) for the reference call sites:

  process_spectrum_from_chunk   preprocessing/preprocess.py:47-49   log1p(|stft|^2)
  melspectrogram                tests/plot_spec.py:20               slaney mel (128) @ |stft|^2
  griffinlim                    model/inference.py:105-110,          momentum 0.99, init random/ones
                                tests/test_griffinlim.py:23
  multi-scale spectral loss     README.md:23, stub model/train.py:119-123 (not implemented in the
                                reference; definition owned by this build: parity unpinned)

Cross-checked against torch.stft/torch.istft (independent pocketfft path) in tests.
"""
import numpy as np


def hann(n):
    """scipy.signal.get_window('hann', n, fftbins=True): periodic Hann, float64."""
    k = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * k / n)


def stft(y, n_fft=2048, hop=256, center=True, pad_mode="reflect", out_dtype=np.complex64):
    """librosa.stft: (1 + n_fft//2, 1 + len(y)//hop) complex64 (float64 math)."""
    y = np.asarray(y)
    if center:
        y = np.pad(y, n_fft // 2, mode=pad_mode)
    n_frames = 1 + (len(y) - n_fft) // hop
    idx = np.arange(n_fft)[None, :] + hop * np.arange(n_frames)[:, None]
    frames = y[idx].astype(np.float64) * hann(n_fft)[None, :]
    X = np.fft.rfft(frames, axis=1).T
    return X.astype(out_dtype) if out_dtype is not None else X


def logpow(y, n_fft=2048, hop=256, pad_mode="reflect"):
    """process_spectrum_from_chunk (preprocess.py:47-49): np.log1p(np.abs(spec)**2), float32."""
    X = stft(y, n_fft, hop, pad_mode=pad_mode)
    return np.log1p(np.abs(X) ** 2)


def hz_to_mel(f):
    f = np.asarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-300) / min_log_hz) / logstep, mels)


def mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def mel_filter(sr, n_fft=2048, n_mels=128, fmin=0.0, fmax=None):
    """librosa.filters.mel(htk=False, norm='slaney') -> (n_mels, 1 + n_fft//2) float32."""
    if fmax is None:
        fmax = sr / 2.0
    nb = 1 + n_fft // 2
    fftfreqs = np.linspace(0, sr / 2.0, nb)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(fmin), hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fftfreqs[None, :]
    w = np.zeros((n_mels, nb), dtype=np.float64)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0, np.minimum(lower, upper))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return w.astype(np.float32)


def melspec(y, sr, n_fft=2048, hop=256, n_mels=128):
    """librosa.feature.melspectrogram (power 2): mel_basis @ |stft|^2 (float64 restatement)."""
    S = np.abs(stft(y, n_fft, hop)).astype(np.float64) ** 2
    return (mel_filter(sr, n_fft, n_mels).astype(np.float64) @ S)


def window_sumsquare(n_frames, n_fft=2048, hop=256):
    n = n_fft + hop * (n_frames - 1)
    x = np.zeros(n, dtype=np.float64)
    w2 = hann(n_fft) ** 2
    for i in range(n_frames):
        s = i * hop
        x[s:min(n, s + n_fft)] += w2[:max(0, min(n_fft, n - s))]
    return x


def istft(X, hop=256, center=True):
    """librosa.istft: windowed irfft overlap-add / window-sum-square, center-trimmed."""
    X = np.asarray(X)
    n_fft = 2 * (X.shape[0] - 1)
    n_frames = X.shape[1]
    frames = np.fft.irfft(X.astype(np.complex128), n=n_fft, axis=0) * hann(n_fft)[:, None]
    y = np.zeros(n_fft + hop * (n_frames - 1), dtype=np.float64)
    for k in range(n_frames):
        y[k * hop:k * hop + n_fft] += frames[:, k]
    wss = window_sumsquare(n_frames, n_fft, hop)
    nz = wss > np.finfo(np.float32).tiny
    y[nz] /= wss[nz]
    if center:
        y = y[n_fft // 2:-(n_fft // 2)]
    return y


def griffinlim(S, n_iter=60, hop=256, momentum=0.99, angles=None, return_all=False):
    """librosa.griffinlim: returns the signal (and optionally each iteration's rebuilt STFT).

    `angles` is the initial unit-phase array (complex); None means all ones
    (init=None). The reference's init='random' is unseeded (inference.py:110);
    callers pass seeded angles for determinism.
    """
    S = np.asarray(S, dtype=np.float64)
    n_fft = 2 * (S.shape[0] - 1)
    a = np.ones(S.shape, dtype=np.complex128) if angles is None else np.asarray(angles, np.complex128)
    rebuilt = 0.0
    hist = []
    for _ in range(n_iter):
        tprev = rebuilt
        inv = istft(S * a, hop)
        rebuilt = stft(inv, n_fft, hop, out_dtype=None)
        a = rebuilt - (momentum / (1 + momentum)) * tprev
        a = a / (np.abs(a) + 1e-16)
        if return_all:
            hist.append(rebuilt)
    y = istft(S * a, hop)
    return (y, hist) if return_all else y


def logpow_to_mag(spec):
    """AudioSynthesizer.griffinlim's inversion (inference.py:109): sqrt(expm1(clip(S, 0, 20)))."""
    return np.sqrt(np.expm1(np.clip(np.asarray(spec, np.float64), 0, 20)))


MSS_SIZES = (2048, 1024, 512, 256, 128, 64)


def multiscale_spectral_loss(pred, target, alpha=1.0, eps=1e-7, sizes=MSS_SIZES):
    """DDSP multi-scale spectral loss (README.md:23; stub train.py:119-123), build definition:

    sum_n  mean|S_n(pred) - S_n(target)| + alpha * mean|log(S_n(pred)+eps) - log(S_n(target)+eps)|
    with S_n = |stft(., n_fft=n, hop=n/4)| (Hann, center, reflect). Parity unpinned.
    pred/target: (L,) or (B, L); the means run over every (clip, bin, frame).
    """
    return multiscale_spectral_loss_grad(pred, target, alpha, eps, sizes, need_grad=False)[0]


def _reflect_index(L, n):
    i = np.arange(L + n) - n // 2
    i = np.where(i < 0, -i, i)
    return np.where(i >= L, 2 * (L - 1) - i, i)


def multiscale_spectral_loss_grad(pred, target, alpha=1.0, eps=1e-7, sizes=MSS_SIZES,
                                  need_grad=True):
    """(loss, d loss / d pred) of multiscale_spectral_loss, by hand (float64):

    dL/dS_n = sign(S_p - S_t) (1 + alpha/(S_p + eps)) / (B F_n T_n)   [sign(log a - log b) = sign(a - b)]
    dL/dX   = dL/dS * X/|X|   (0 where |X| = 0, as torch.abs' subgradient)
    frame gradient r_j = Re sum_{f=0}^{n/2} dL/dX_f e^{+2 pi i f j/n}, times the window,
    overlap-added into the padded signal and folded back through the reflect padding.
    Cross-checked against torch float64 autograd (tests/test_cpu_oracle.py).
    """
    P = np.atleast_2d(np.asarray(pred, dtype=np.float64))
    Q = np.atleast_2d(np.asarray(target, dtype=np.float64))
    B, L = P.shape
    total = 0.0
    dP = np.zeros_like(P) if need_grad else None
    for n in sizes:
        h = n // 4
        T = 1 + L // h
        N = n // 2
        w = hann(n)
        ridx = _reflect_index(L, n)
        fidx = np.arange(n)[None, :] + h * np.arange(T)[:, None]       # (T, n) padded positions
        Xp = np.fft.rfft(P[:, ridx][:, fidx] * w, axis=2)               # (B, T, N+1)
        Xt = np.fft.rfft(Q[:, ridx][:, fidx] * w, axis=2)
        Sp, St = np.abs(Xp), np.abs(Xt)
        cnt = B * T * (N + 1)
        total += np.abs(Sp - St).sum() / cnt + alpha * np.abs(np.log(Sp + eps) - np.log(St + eps)).sum() / cnt
        if not need_grad:
            continue
        G = np.sign(Sp - St) * (1.0 + alpha / (Sp + eps)) / cnt
        U = np.divide(Xp, Sp, out=np.zeros_like(Xp), where=Sp > 0)
        Z = np.zeros((B, T, n), dtype=np.complex128)
        Z[:, :, :N + 1] = G * U
        r = np.real(np.fft.ifft(Z, axis=2)) * n * w                    # (B, T, n)
        dpad = np.zeros((B, L + n))
        for t in range(T):
            dpad[:, t * h:t * h + n] += r[:, t]
        for b in range(B):
            np.add.at(dP[b], ridx, dpad[b])
    if need_grad and np.ndim(pred) == 1:
        dP = dP[0]
    return total, dP
