"""Deterministic, framework-independent tensors for parity tests.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): imported by tests/, bench.py's
cpu_baseline leg and __graft_entry__.smoke(); never by the product package.

Every value is a pure function of (name, flat index) through a splitmix64 hash,
so the golden-fixture generator (which imports the reference model in the build
container) and the GPU tests (which run without /root/reference) build
bit-identical weights and inputs without shipping them as files.
"""
import zlib

import numpy as np

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_GOLD = np.uint64(0x9E3779B97F4A7C15)


def _splitmix64(x):
    with np.errstate(over="ignore"):
        z = x + _GOLD
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(name, shape, lo=-1.0, hi=1.0, seed=0):
    """float32 array in [lo, hi), deterministic in (seed, name, index)."""
    n = int(np.prod(shape)) if len(shape) else 1
    key = np.uint64((zlib.crc32(name.encode()) << 20) ^ (seed & 0xFFFFF))
    idx = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = _splitmix64(idx * np.uint64(0x100000001B3) + (key << np.uint64(24)))
    u = (h >> np.uint64(40)).astype(np.float64) / float(1 << 24)  # [0,1) with 24 bits
    return (lo + (hi - lo) * u).astype(np.float32).reshape(shape)


def randint(name, shape, lo, hi, seed=0):
    """int64 array in [lo, hi)."""
    u = uniform(name, shape, 0.0, 1.0, seed).astype(np.float64)
    return np.minimum(lo + np.floor(u * (hi - lo)).astype(np.int64), hi - 1)


def param_value(name, shape, seed=0):
    """Deterministic stand-in for PerformanceNet's init (model.py:249-260).

    Conv/ConvT weights: uniform with the xavier_normal_ standard deviation;
    Linear weights: torch's default kaiming-uniform bound 1/sqrt(fan_in);
    biases: small non-zero values so the bias paths are exercised.
    """
    shape = tuple(shape)
    if name.endswith("bias"):
        return uniform(name, shape, -0.05, 0.05, seed)
    if len(shape) == 3:  # Conv1d (out,in,k) or ConvTranspose1d (in,out,k)
        rf = shape[2]
        fan_in, fan_out = shape[1] * rf, shape[0] * rf
        std = (2.0 / (fan_in + fan_out)) ** 0.5
        b = std * 3.0 ** 0.5
        return uniform(name, shape, -b, b, seed)
    if len(shape) == 2:  # Linear (out, in)
        b = 1.0 / shape[1] ** 0.5
        return uniform(name, shape, -b, b, seed)
    return uniform(name, shape, -0.1, 0.1, seed)


def model_inputs(B, T, seed=0, n_pitch=128, n_bins=1025):
    """Synthetic (x_midi {0,1}, x_audio log-power, cond {-1,0,1}, target) in NCL."""
    x_midi = (uniform("x_midi", (B, n_pitch, T), 0, 1, seed) < 0.1).astype(np.float32)
    cond = randint("cond", (B, n_pitch, T), -1, 2, seed).astype(np.float32)
    cond *= (uniform("cond_mask", (B, n_pitch, T), 0, 1, seed) < 0.05)
    x_audio = uniform("x_audio", (B, n_bins, T), 0.0, 4.0, seed) ** 2 / 4.0
    target = uniform("target", (B, n_bins, T), 0.0, 4.0, seed) ** 2 / 4.0
    return x_midi, x_audio, cond.astype(np.float32), target


def offgrid_target(B, T_out, seed=0, n_bins=1025):
    """L1 target for an input length T whose output length T_out = 16 * floor(T / 16) + 12
    differs from T (model.py:229-232): drawn at the output's length."""
    return uniform("target_offgrid", (B, n_bins, T_out), 0.0, 4.0, seed) ** 2 / 4.0
