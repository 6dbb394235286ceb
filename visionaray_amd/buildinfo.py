"""Identity of the kernel build a measurement belongs to: the SHA-256 of the sources libvrh's kernels
are compiled from (visionaray_amd/csrc, include/vrh.h, include/visionaray_hip/detail/vrh_device.h).
tools/pmc_bench.py stores it in every committed PMC pass; bench.py reports the pass's counters only
when the running tree has the same hash (a stale pass would report stale achieved / frac)."""
import glob
import hashlib
import os

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_sources():
    files = sorted(glob.glob(os.path.join(_ROOT, "visionaray_amd", "csrc", "*.hip"))
                   + glob.glob(os.path.join(_ROOT, "visionaray_amd", "csrc", "*.h"))
                   + glob.glob(os.path.join(_ROOT, "visionaray_amd", "csrc", "*.cpp")))
    return files + [os.path.join(_ROOT, "include", "vrh.h"),
                    os.path.join(_ROOT, "include", "visionaray_hip", "detail", "vrh_device.h")]


def _sha256(files):
    h = hashlib.sha256()
    for p in files:
        h.update(os.path.relpath(p, _ROOT).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def kernel_source_sha256():
    return _sha256(kernel_sources())


def user_kernel_sources():
    """The user-kernel programs' sources on top of libvrh's: the device headers they are compiled from
    (include/visionaray_hip) and the test program the bench's user leg runs."""
    return (kernel_sources() + sorted(glob.glob(os.path.join(_ROOT, "include", "visionaray_hip", "*.h"))
                                      + glob.glob(os.path.join(_ROOT, "include", "visionaray_hip", "detail", "*.h")))
            + [os.path.join(_ROOT, "tests", "cpp", "user_kernels.hip")])


def user_kernel_source_sha256():
    return _sha256(user_kernel_sources())
