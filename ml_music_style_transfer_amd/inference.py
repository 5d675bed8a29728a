"""Drop-in for the reference synthesis path (model/inference.py) on the device.

`AudioSynthesizer.griffinlim` keeps the reference signature (inference.py:105-110):
log-power in, sqrt(expm1(clip(S,0,20))) magnitude, librosa.griffinlim with
momentum 0.99 — here one fused device program (iSTFT -> STFT -> momentum per
iteration, fft.hip). The reference's init='random' is unseeded; `seed` fixes it.
MIDI parsing, librosa.load and soundfile output (inference.py:37-72,91,112-124)
are file I/O outside the hot path; `synthesize` runs model forward + Griffin-Lim
for tensors already in memory.
"""
import numpy as np
import torch

from . import spectral
from .model import PerformanceNet
from .preprocess import hp as pp_hp


class AudioSynthesizer():
    """inference.py:22-110 (compute parts)."""

    def __init__(self, checkpoint=None, exp_dir=None, midi_source=None, audio_source=None):
        self.exp_dir = exp_dir
        self.checkpoint = checkpoint
        self.sample_rate = pp_hp.sr
        self.wps = pp_hp.wps
        self.midi_source = midi_source
        self.audio_source = audio_source

    def griffinlim(self, spectrogram, audio_id, n_iter=300, window='hann', n_fft=2048,
                   hop_length=256, verbose=False, seed=0):
        """inference.py:105-110. spectrogram: (1025, T) log-power (NumPy or tensor)."""
        if window != 'hann' or n_fft != 2048:
            raise ValueError("the reference path uses a 2048-point Hann window")
        is_np = not isinstance(spectrogram, torch.Tensor)
        S = torch.from_numpy(np.ascontiguousarray(spectrogram, np.float32)) if is_np else spectrogram
        S = S.cuda() if not S.is_cuda else S
        y = spectral.griffinlim(S.float(), n_iter=n_iter, hop_length=hop_length, momentum=0.99,
                                init="random", seed=seed, from_logpow=True)
        return y.cpu().numpy() if is_np else y

    def synthesize(self, model, score, spec, onoff, n_iter=300, seed=0):
        """model forward (no_grad, eval) then Griffin-Lim of every item (inference.py:74-91)."""
        with torch.no_grad():
            model.eval()
            out = model(score, spec, onoff)
        return spectral.griffinlim(out, n_iter=n_iter, momentum=0.99, init="random", seed=seed,
                                   from_logpow=True)


__all__ = ["AudioSynthesizer", "PerformanceNet"]
