"""The device build of detail/vrh_libm.h (glibc's sinf / cosf restated) equals its host build -- which
equals the host C library on every float input (tests/test_libm_sincosf.py) -- bit for bit: every float
of the sampler's argument range [0, 2 pi) and a strided sample of all 2^32 bit patterns
(build/tests/libm_check, tests/cpp/libm_check.hip)."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "tests", "libm_check")

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("lo,hi,stride", [(0, 0x40C90FDB, 1), (0, 1 << 32, 251)])
def test_device_sincosf_equal_host(lo, hi, stride):
    out = subprocess.run([BIN, str(lo), str(hi), str(stride)], capture_output=True, text=True, timeout=110)
    r = json.loads(out.stdout)
    assert out.returncode == 0 and r["device_vs_host_restatement"] == 0, r
    if r["host_fma"] and r["host_avx2"]:
        assert r["device_vs_host_libm"] == 0, r
