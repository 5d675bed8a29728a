"""The measured numbers the bench line quotes from profiles/ (CPU): the GEMM PMC summary and every
HBM-traffic figure name the tracked commit they were measured on, and
bench.py's readers return them in the form the line carries.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _commit_of(label):
    m = re.search(r"commit ([0-9a-f]{7,40})", label or "")
    assert m, f"no commit named in {label!r}"
    return m.group(1)


def _in_history(h):
    if not os.path.isdir(os.path.join(ROOT, ".git")):
        pytest.skip("no git history here")
    r = subprocess.run(["git", "cat-file", "-e", f"{h}^{{commit}}"], cwd=ROOT, capture_output=True)
    return r.returncode == 0


def test_gemm_pmc_and_traffic_name_their_commit():
    import bench
    pmc = bench.gemm_pmc()
    assert pmc is not None and set(pmc["kinds"]) >= {"conv", "dgrad", "wgrad"}
    for k in ("conv", "dgrad", "wgrad"):
        e = pmc["kinds"][k]
        assert 0 < e["mfma_busy"] < 1 and e["valu_per_mfma"] > 0 and "counters" not in e
    assert _in_history(_commit_of(pmc["build"]))
    traffic, src = bench.gemm_traffic()
    assert traffic and traffic > 0
    assert _in_history(_commit_of(src))


def test_aux_traffic_sources_name_their_commit():
    import bench_aux
    for traffic, src in (bench_aux._measured_traffic("stft_fm_kernel<0,"),
                         bench_aux._measured_traffic("stft_fm_kernel<2,"),
                         bench_aux._gl_traffic(60), bench_aux._mss_traffic()):
        assert traffic and traffic > 0, src
        assert _in_history(_commit_of(src)), src
