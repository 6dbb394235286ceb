"""include/visionaray_hip/detail/vrh_libm.h restates the host C library's sinf / cosf (glibc 2.35, the
FMA variants x86_64 selects on this container's CPU) so that the reference's cosine_sample_hemisphere
(sampling.h:61-71) draws the same directions on the device as on the CPU.  Here: the host build of the
restatement against the host library on EVERY float input (2^32 bit patterns, both functions; NaN
results compare as NaN), with and without floating-point contraction.  The device build is checked
against the host build on the GPU (tests/test_gpu_libm.py)."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "libm_check.cpp")


def _build(tmp_path, contract):
    exe = tmp_path / f"libm_check_{contract}"
    subprocess.run(["g++", "-O2", "-std=c++17", f"-ffp-contract={contract}", "-pthread",
                    "-I", os.path.join(ROOT, "include"), SRC, "-o", str(exe)], check=True)
    return exe


def _run(exe, lo, hi):
    out = subprocess.run([str(exe), str(lo), str(hi), str(min(8, os.cpu_count() or 1))],
                         capture_output=True, text=True, timeout=600)
    return json.loads(out.stdout)


def test_every_float_input_matches_host_libm(tmp_path):
    r = _run(_build(tmp_path, "off"), 0, 1 << 32)
    if not (r["fma"] and r["avx2"]):
        pytest.skip("this CPU makes glibc select its SSE2 sinf / cosf, not the FMA variants restated")
    assert r["inputs"] == 1 << 32
    assert r["sinf_mismatch"] == 0 and r["cosf_mismatch"] == 0, r


def test_sampler_range_matches_with_contraction(tmp_path):
    """[0, 2 pi): the arguments cosine_sample_hemisphere passes (two_pi * u2, u2 in [0, 1)), built with
    -ffp-contract=fast: no plain product in the header feeds an addition, so nothing is fused."""
    r = _run(_build(tmp_path, "fast"), 0, 0x40C90FDB)
    if not (r["fma"] and r["avx2"]):
        pytest.skip("this CPU makes glibc select its SSE2 sinf / cosf")
    assert r["sinf_mismatch"] == 0 and r["cosf_mismatch"] == 0, r
