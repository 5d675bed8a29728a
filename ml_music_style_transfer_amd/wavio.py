"""WAV input/output on either side of the synthesis path.

The reference loads audio with `librosa.load(path, sr=44100)` (preprocess.py:106,
inference.py:54) and writes with `soundfile.write(path, audio, sr)`
(inference.py:91). Neither library is in this image; this module restates the
parts the path uses with the standard library (parity unpinned):

- read: PCM 8/16/24/32-bit and IEEE float32/64 WAV, scaled as libsndfile reads
  to float (int / 2^(bits-1); 8-bit is unsigned), averaged to mono
  (librosa.to_mono), float32. librosa resamples a file whose rate differs from
  `sr` (resampy/soxr filters); that filter is not restated, so a rate mismatch
  raises instead of silently changing the signal.
- write: soundfile's default WAV subtype for float data, PCM_16, with
  libsndfile's float->short scale 0x7FFF, round to nearest, clipped.
"""
import struct
import wave

import numpy as np

__all__ = ["load", "write"]


def _read_raw(path):
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError("not a RIFF/WAVE file: %s" % path)
    i, fmt, body = 12, None, None
    while i + 8 <= len(data):
        cid, ln = data[i:i + 4], struct.unpack("<I", data[i + 4:i + 8])[0]
        chunk = data[i + 8:i + 8 + ln]
        if cid == b"fmt ":
            fmt = struct.unpack("<HHIIHH", chunk[:16])
            if fmt[0] == 0xFFFE and len(chunk) >= 26:  # WAVE_FORMAT_EXTENSIBLE: subformat tag
                fmt = (struct.unpack("<H", chunk[24:26])[0],) + fmt[1:]
        elif cid == b"data":
            body = chunk
        i += 8 + ln + (ln & 1)
    if fmt is None or body is None:
        raise ValueError("WAV without fmt/data chunk: %s" % path)
    tag, nch, sr, _, _, bits = fmt
    if (tag == 3 and bits not in (32, 64)) or (tag == 1 and bits not in (8, 16, 24, 32)):
        raise ValueError("unsupported WAV sample width: %d bits (format %d)" % (bits, tag))
    if tag == 3:
        x = np.frombuffer(body, dtype={32: "<f4", 64: "<f8"}[bits]).astype(np.float64)
    elif tag == 1:
        if bits == 8:
            x = (np.frombuffer(body, np.uint8).astype(np.float64) - 128.0) / 128.0
        elif bits == 24:
            b = np.frombuffer(body, np.uint8).reshape(-1, 3).astype(np.int32)
            v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
            v = np.where(v & 0x800000, v - (1 << 24), v)
            x = v.astype(np.float64) / float(1 << 23)
        else:
            x = np.frombuffer(body, {16: "<i2", 32: "<i4"}[bits]).astype(np.float64) / float(1 << (bits - 1))
    else:
        raise ValueError("unsupported WAV format tag %d" % tag)
    n = len(x) // nch
    return x[:n * nch].reshape(n, nch), sr


def load(path, sr=44100, mono=True):
    """librosa.load(path, sr=sr, mono=mono) -> (y float32, sr)."""
    x, file_sr = _read_raw(path)
    if sr is not None and file_sr != sr:
        raise ValueError("%s is %d Hz, expected %d Hz (resampling is not restated)"
                         % (path, file_sr, sr))
    y = x.mean(axis=1) if mono else x.T
    return y.astype(np.float32), file_sr


def write(path, audio, samplerate):
    """soundfile.write(path, audio, samplerate) for float audio -> 16-bit PCM WAV."""
    a = np.asarray(audio, dtype=np.float64)
    if a.ndim == 1:
        a = a[:, None]
    pcm = np.clip(np.rint(a * 32767.0), -32768, 32767).astype("<i2")
    with wave.open(path, "wb") as w:
        w.setnchannels(a.shape[1])
        w.setsampwidth(2)
        w.setframerate(int(samplerate))
        w.writeframes(pcm.tobytes())
