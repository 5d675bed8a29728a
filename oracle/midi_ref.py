"""Integer framing / chunking / piano-roll restatement — parity oracle (bit-exact rules).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

  hyperparams framing   preprocessing/preprocess.py:17-42   sr, n_fft, ws(hop), wps=sr//ws, spc, stride
  audio chunk slice     preprocess.py:66-67                 audio[step*ws*stride : +(spc*wps-1)*ws]
  roll chunk slice      preprocess.py:86-88                 roll[step*stride : +spc*wps]
  get_num_song_chunks   preprocess.py:118-136               (n - spc*wps)//stride, minus int(0.1*.), cap
  load_midi roll/onoff  preprocess.py:146-155               pretty_midi get_piano_roll(fs=wps).T, binarise,
                                                            onoff row i = +1 on new notes, -1 on released
  batch assembly        model/train.py:82-85,130            concat(roll, onoff).T, split at 128
pretty_midi is absent here: get_piano_roll is restated from its published
algorithm (roll[pitch, int(start*fs):int(end*fs)] += velocity, no sustain
pedal events in synthetic notes) — parity unpinned against pretty_midi itself.
"""
import numpy as np


class Hyper:
    def __init__(self, sr=44100, n_fft=2048, ws=256, spc=5, stride=512):
        self.sr, self.n_fft, self.ws, self.spc, self.stride = sr, n_fft, ws, spc, stride
        self.wps = sr // ws


def audio_chunk_bounds(hp, step):
    n = (hp.spc * hp.wps - 1) * hp.ws
    s = step * hp.ws * hp.stride
    return s, s + n


def roll_chunk_bounds(hp, step):
    n = hp.spc * hp.wps
    s = step * hp.stride
    return s, s + n


def num_song_chunks(n_windows, hp, offset_percentage=0.1, max_chunks=100):
    num = (n_windows - hp.spc * hp.wps) // hp.stride
    num -= int(offset_percentage * num)
    return min(num, max_chunks)


def piano_roll(notes, fs, n_frames=None):
    """notes: iterable of (pitch, start_s, end_s, velocity) -> (128, n) float like pretty_midi."""
    notes = list(notes)
    end = max((n[2] for n in notes), default=0.0)
    n = int(fs * end) if n_frames is None else n_frames
    roll = np.zeros((128, n), dtype=np.float64)
    for p, s, e, v in notes:
        roll[int(p), int(s * fs):int(e * fs)] += v
    return roll


def binarize_and_onoff(roll_T):
    """roll_T: (frames, 128). Returns binarised roll and onoff exactly as preprocess.py:148-155."""
    pr = np.array(roll_T, dtype=np.float64, copy=True)
    pr[pr.nonzero()] = 1
    onoff = np.zeros(pr.shape)
    for i in range(pr.shape[0]):
        if i == 0:
            onoff[i][pr[i].nonzero()] = 1
        else:
            onoff[i][np.setdiff1d(pr[i - 1].nonzero(), pr[i].nonzero())] = -1
            onoff[i][np.setdiff1d(pr[i].nonzero(), pr[i - 1].nonzero())] = 1
    return pr, onoff


def assemble_item(roll_chunk, onoff_chunk):
    """Dataseth5py.__getitem__ lines 82-85: concat on last axis then transpose -> (256, T)."""
    return np.transpose(np.concatenate((roll_chunk, onoff_chunk), axis=-1), (1, 0))
