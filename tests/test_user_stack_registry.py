"""The depth registry behind the user kernels' short LDS stacks (include/visionaray_hip/hip_backend.h
note_ref_depth / user_ref_depth): a launch gives each thread VRH_USER_LDS_STACK entries only while every
BVH the program has taken a ref of is shallower, so the registry must never lose a deeper depth --
checked single-threaded and with 8 threads noting depths at once (host code, g++)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_ref_depth_registry_keeps_the_maximum(tmp_path):
    exe = tmp_path / "ref_depth_registry"
    subprocess.run(["g++", "-std=c++17", "-O2", "-pthread", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "ref_depth_registry.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip() == "ok 30"
