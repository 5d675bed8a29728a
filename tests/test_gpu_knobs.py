"""The A/B knobs that stay in the library each switch a kernel path off its
measured default. They are read once per process, so every setting runs tests/_knob_child.py in
a child process (one at a time) and its outputs are compared with this process's default-build
results: GEMMs within 2e-5 of the absolute-product scale (the variants sum in another order),
InstanceNorm within 2e-5 (as test_gpu_kernels.py), Adam within 1e-6 absolute (same arithmetic,
another launch shape), Griffin-Lim within 1e-5 of the signal's peak (other workgroup seams: the
two partial sums of a seam sample are rounded at other places).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

KNOBS = [
    {"MST_GEMM_WIDE": "0"},         # conv / dgrad on the 128 x 128 kernel
    {"MST_GEMM_SCHED": "sk"},       # stream-K for every GEMM
    {"MST_SPLITK_TAU": "1e-9"},     # split-K cost model pushed to no split
    {"MST_SLAB4": "0"},             # split-K slabs stored element by element
    {"MST_REDUCE_ROWS": "0"},       # split-K reduce as a 1-D float4 grid (a division per element)
    {"MST_WG_TWO": "0"},            # k3 wgrad B planes in three tap copies instead of two
    {"MST_WG_PLANES": "0"},         # wgrad on the register-split 128 x 128 kernel (K classes)
    {"MST_WG_PLANES": "0", "MST_WG_VEC": "0"},  # ... with dword loads in the unmasked classes too
    {"MST_IN_SEG": "0"},            # one InstanceNorm row per wave
    {"MST_ADAM_VARIANT": "1p"},     # Adam: one float4 group per thread, plain loads/stores
    {"MST_GL_FRAMES": "8", "MST_GL_CHUNK_MB": "1"},  # Griffin-Lim: 8-frame workgroups, 1-clip chunks
]

def _tol(key, ref):
    if key.startswith("deep_") or key.startswith("wide_"):
        B, Cin, Cout, T = (32, 512, 512, 15) if key.startswith("deep_") else (4, 96, 130, 252)
        scale = {"fwd": Cin * 3, "dgrad": Cout * 3, "wgrad": B * T}[key.split("_")[1]]
        return 2e-5 * scale
    if key.startswith("in"):
        return 2e-5 * (int(key[2:].split("_")[0]) if key.endswith("_rs") else 10)
    if key == "gl":
        return 1e-5 * float(np.max(np.abs(ref)))
    return 1e-6


@pytest.fixture(scope="module")
def default_outputs(cuda):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _knob_child
    return _knob_child.run(cuda)


@pytest.mark.timeout(240)
@pytest.mark.parametrize("knob", KNOBS, ids=lambda k: ",".join(f"{a}={b}" for a, b in k.items()))
def test_knob_matches_default(default_outputs, knob, tmp_path):
    out = tmp_path / "knob.npz"
    env = dict(os.environ, **knob)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "_knob_child.py"), str(out)],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-3000:]
    got = np.load(out)
    assert set(got.files) == set(default_outputs)
    for k, ref in default_outputs.items():
        err = float(np.max(np.abs(got[k].astype(np.float64) - ref.astype(np.float64))))
        tol = _tol(k, ref)
        assert err <= tol, f"{knob}: {k} differs from the default by {err:.3e} > {tol:.3e}"
