"""Drop-in for the reference front end (preprocessing/preprocess.py), on the device.

`process_spectrum_from_chunk` keeps the reference signature and returns the
same (1025, 1 + L//256) float32 array type it was given (NumPy in -> NumPy out,
CUDA tensor in -> CUDA tensor out); the STFT itself always runs in libmst_hip.
The integer chunk/frame arithmetic is the reference's, bit for bit.
`load_midi` / `load_audio` / `get_data` / `main` (preprocess.py:99-215) keep the
reference's signatures: file globbing as the reference, pretty_midi and librosa.load
restated in midi.py / wavio.py, HDF5 written through h5.py.
"""
import glob

import os

import numpy as np
import torch

from . import ops as _ops  # noqa: F401  (registers torch.ops.mst.*)
from . import spectral


class hyperparams(object):
    """preprocess.py:17-42 (framing constants)."""

    def __init__(self, sr=44100, n_fft=2048, stride=512, ws=256, spc=5):
        self.sr = sr
        self.n_fft = n_fft
        self.stride = stride
        self.piano_scores = {
            'train': [2240, 2530, 1763, 2308, 2533, 1772, 2444, 2478,
                      2509, 1776, 1749, 2486, 2487, 2678, 2490, 2492, 2527],
            'test': [2533, 1760],
        }
        self.styles = ['cuba', 'aliciakeys', 'gentleman', 'harpsichord', 'upright']
        self.ws = ws
        self.wps = self.sr // self.ws
        self.spc = spc


hp = hyperparams()


def _to_device(x):
    if isinstance(x, torch.Tensor):
        return (x if x.is_cuda else x.cuda()).float(), "torch_cuda" if x.is_cuda else "torch_cpu"
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).cuda(), "numpy"


def _back(t, kind):
    if kind == "numpy":
        return t.cpu().numpy()
    if kind == "torch_cpu":
        return t.cpu()
    return t


def process_spectrum_from_chunk(audio_chunk, hop=None, pad_mode="reflect"):
    """preprocess.py:47-49: log1p(|stft(audio_chunk, n_fft=2048, hop_length=256)|^2).
    Accepts (L,) or a batch (B, L)."""
    x, kind = _to_device(audio_chunk)
    out = spectral.stft_logpow(x, hop=hop or hp.ws, n_fft=hp.n_fft, pad_mode=pad_mode)
    return _back(out, kind)


def chunk_bounds_audio(step, h=hp):
    """preprocess.py:66-67."""
    n = (h.spc * h.wps - 1) * h.ws
    s = step * h.ws * h.stride
    return s, s + n


def chunk_bounds_roll(step, h=hp):
    """preprocess.py:86-87."""
    n = h.spc * h.wps
    s = step * h.stride
    return s, s + n


def process_audio_into_chunks(audio, style, song_id, num_chunks, debug=False, h=hp):
    """preprocess.py:60-77, with every chunk's STFT batched into one kernel launch."""
    print(f"processing {style} style for song_id {song_id}")
    x, kind = _to_device(audio)
    chunks = []
    for step in range(num_chunks):
        s, e = chunk_bounds_audio(step, h)
        chunks.append(x[s:e])
    if not chunks:
        return np.zeros((0,)) if kind == "numpy" else torch.zeros(0)
    n = (h.spc * h.wps - 1) * h.ws
    if all(c.shape[0] == n for c in chunks):
        out = spectral.stft_logpow(torch.stack(chunks), hop=h.ws, n_fft=h.n_fft)
        return _back(out, kind)
    outs = [spectral.stft_logpow(c, hop=h.ws, n_fft=h.n_fft) for c in chunks]  # ragged tail
    return np.array([_back(o, kind) for o in outs], dtype=object) if kind == "numpy" else outs


def process_pianoroll_into_chunks(pianoroll, onoff, song_id, num_chunks, debug=False, h=hp):
    """preprocess.py:80-96 (pure slicing)."""
    print(f"processing pianoroll for song_id {song_id}")
    score_list, onoff_list = [], []
    for step in range(num_chunks):
        s, e = chunk_bounds_roll(step, h)
        score_list.append(pianoroll[s:e])
        onoff_list.append(onoff[s:e])
    return np.array(score_list), np.array(onoff_list)


def get_num_song_chunks(pianoroll, offset_percentage=0.1, max_chunks=100, h=hp):
    """preprocess.py:118-136."""
    n_windows_per_chunk = h.spc * h.wps
    num_chunks = (pianoroll.shape[0] - n_windows_per_chunk) // h.stride
    offset = int(offset_percentage * num_chunks)
    num_chunks -= offset
    if num_chunks > max_chunks:
        print(f"song has more than max_chunks={max_chunks}, reducing")
        num_chunks = max_chunks
    print('song has {} chunks'.format(num_chunks))
    return num_chunks


def pianoroll_onoff(roll):
    """preprocess.py:147-155 on the device: roll (T, 128) or (B, T, 128) velocities ->
    (binarised roll, onoff) with onoff[t] = roll[t] - roll[t-1] in {-1, 0, 1}."""
    x, kind = _to_device(roll)
    single = x.dim() == 2
    if single:
        x = x.unsqueeze(0)
    x = x.contiguous()
    B, T, P = x.shape
    if P != 128:
        raise ValueError("piano roll must have 128 pitches on the last axis")
    b, o = torch.ops.mst.onoff(x)
    if single:
        b, o = b[0], o[0]
    return _back(b, kind), _back(o, kind)


def piano_roll_from_notes(notes, fs, n_frames=None):
    """pretty_midi.PrettyMIDI.get_piano_roll(fs) for a note list (pitch, start_s, end_s, velocity)
    without sustain-pedal events (preprocess.py:147): (128, n) float64."""
    notes = list(notes)
    end = max((n[2] for n in notes), default=0.0)
    n = int(fs * end) if n_frames is None else n_frames
    roll = np.zeros((128, n), dtype=np.float64)
    for p, s, e, v in notes:
        roll[int(p), int(s * fs):int(e * fs)] += v
    return roll



def midi_file_to_roll(midi_path, h=hp, pedal_threshold=64):
    """The body of preprocess.py:146-155 for one file: pretty_midi piano roll at wps frames/s
    (restated in midi.py), then the binarised roll and onoff on the device. Returns float64
    (T, 128) arrays like the reference."""
    from . import midi as _midi
    roll = _midi.get_piano_roll(midi_path, fs=h.wps, pedal_threshold=pedal_threshold).T
    if roll.shape[0] == 0:
        return np.zeros((0, 128)), np.zeros((0, 128))
    b, o = pianoroll_onoff(roll)
    return b.astype(np.float64), o.astype(np.float64)


def read_audio(audio_path, h=hp):
    """librosa.load(path, sr=hp.sr) (preprocess.py:106) via wavio (no resampling)."""
    from . import wavio
    y, _ = wavio.load(audio_path, sr=h.sr)
    return y


def _one_file(pattern, what):
    files = glob.glob(pattern)
    if len(files) == 0:
        raise ValueError("couldnt find %s track!" % what)
    elif len(files) > 1:
        raise ValueError("multiple files picked up, issue:", files)
    return files[0]


def load_audio(data_dir, song_id, style, debug=False, h=hp):
    """preprocess.py:99-115."""
    path = _one_file(f"{data_dir}/{song_id}*{style}.wav", "audio")
    y = read_audio(path, h)
    if debug is True:
        print("length of audio clip / sr: ", len(y), h.sr)
        print("audio files picked up:", [path])
    return y


def load_midi(data_dir, song_id, ext='mixcraft', debug=False, h=hp):
    """preprocess.py:139-160."""
    path = _one_file(f"{data_dir}/{song_id}*{ext}.mid", "midi")
    pianoroll, onoff = midi_file_to_roll(path, h)
    if debug is True:
        print("length of pianoroll: ", pianoroll.shape)
        print("midi files picked up:", [path])
    return pianoroll, onoff


def get_data(data_dir, dataset_outpath, data_type, debug=False, h=hp):
    """preprocess.py:163-200: every song of hp.piano_scores[data_type] -> pianoroll/onoff
    chunks and, per style whose audio exists, log-power spectrogram chunks (one batched STFT
    launch per song and style), appended to `<dataset_outpath>_<data_type>.hdf5`
    (io_manager.h5pyManager layout, data.h5pyManager). Like the reference, a missing style
    is skipped for that song."""
    from . import h5
    from .data import h5pyManager
    h5name = f"{dataset_outpath}_{data_type}.hdf5"
    with h5.File(h5name, 'w') as h5_data:
        manager = h5pyManager(h5_data)
        for song_id in h.piano_scores[data_type]:
            pianoroll, onoff = load_midi(data_dir, song_id, debug=debug, h=h)
            num_chunks = get_num_song_chunks(pianoroll, h=h)
            pianoroll_list, onoff_list = process_pianoroll_into_chunks(pianoroll, onoff, song_id,
                                                                       num_chunks, debug=debug, h=h)
            manager.write_pianoroll(pianoroll_list, onoff_list)
            for style in h.styles:
                try:
                    audio = load_audio(data_dir, song_id, style, debug=debug, h=h)
                except (ValueError, OSError):
                    print(f"Couldnt load audio for song={song_id}, style={style}, skipping...")
                    continue
                spec_list = process_audio_into_chunks(audio, style, song_id, num_chunks,
                                                      debug=debug, h=h)
                manager.write_spectrum(np.asarray(spec_list, dtype=np.float64), style)
    return h5name


def resolve_data_dir(data_dir, extract_to=None):
    """preprocess.py:204-210: a zip `-data-dir` is unpacked into the working directory (or
    `extract_to`) and replaced by the directory of its first member; a directory is returned
    as is."""
    import zipfile
    if not zipfile.is_zipfile(data_dir):
        return data_dir
    print("Extracting zip file to local")
    dest = os.getcwd() if extract_to is None else extract_to
    with zipfile.ZipFile(data_dir) as zf:
        first = zf.namelist()[0]
        zf.extractall(dest)
    return os.path.join(dest, os.path.dirname(first))


def main(args):
    """preprocess.py:203-215: optional zip extraction, then get_data."""
    data_dir = resolve_data_dir(args.data_dir)
    return get_data(data_dir, args.dataset_outpath, args.data_type, args.debug)


def parse_args(argv=None):
    import argparse
    parser = argparse.ArgumentParser()
    parser.add_argument("-data-dir", type=str, required=True,
                        help="dataset directory, or a zip file that is extracted first")
    parser.add_argument("-dataset-outpath", type=str, required=True)
    parser.add_argument("-max-chunks-per-song", type=int, default=100)
    parser.add_argument("-data-type", type=str, default='train', choices=['train', 'test'])
    parser.add_argument("--debug", type=lambda v: str(v).lower() in ('yes', 'true', 't', 'y', '1'),
                        default=False)
    return parser.parse_args(argv)


if __name__ == "__main__":
    main(parse_args())
