import os
import sys

import pytest

# The CPU suite pins the oracle bit-for-bit to fixtures made with MKL's COMPATIBLE code path
# (tests/golden/make_golden.py): it is the one path MKL honours on both Intel and AMD hosts, and it
# must be chosen before the first MKL call of the process. A `-m gpu` run keeps MKL's fast default
# path, because its oracle checks are tolerance-based and run at C2 sizes.
def _gpu_only_run(argv):
    for i, a in enumerate(argv):
        if a == "-m" and i + 1 < len(argv):
            return argv[i + 1].strip() == "gpu"
        if a.startswith("-m") and a[2:].strip() == "gpu":
            return True
    return False


if not _gpu_only_run(sys.argv):
    os.environ.setdefault("MKL_CBWR", "COMPATIBLE")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "genome-minimizer-2_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libgm2.so on cuda:0)")


@pytest.fixture(autouse=True)
def _one_thread():
    """Reference goldens were produced at torch.set_num_threads(1)."""
    import torch
    n = torch.get_num_threads()
    torch.set_num_threads(1)
    yield
    torch.set_num_threads(n)


@pytest.fixture(autouse=True)
def _debug_build_flags(request):
    """Under the debug build (GM2_LIB_PATH=.../libgm2_debug.so, the whole -m gpu suite run against
    it): every kernel check of index data ORs a bit into a device flag word instead of trapping
    (include/gm2_debug.h); after each GPU test the flags are read (and cleared) and must be 0."""
    yield
    if not os.environ.get("GM2_LIB_PATH", "").endswith("libgm2_debug.so") or "gpu" not in request.keywords:
        return
    import ctypes

    import torch
    from gm2 import native
    torch.cuda.synchronize()
    v = ctypes.c_uint(0)
    native.check(native.lib().gm2_debug_flags(ctypes.byref(v)), "gm2_debug_flags")
    assert v.value == 0, f"debug build: index check flags {v.value:#x} after {request.node.nodeid}"
