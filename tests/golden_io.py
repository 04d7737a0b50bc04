"""Loaders for the committed golden fixtures (tests/golden/*.npz, made by make_golden.py)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def meta(g):
    return json.loads(str(g["meta"])) if "meta" in g.files else {}


def host_cpu():
    """The CPU model string make_golden.py records in every fixture's meta."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def same_mkl_path(g):
    """True when this process runs MKL on the code path the fixture was made on.

    make_golden.py fixes MKL_CBWR=COMPATIBLE and tests/conftest.py selects it for the CPU suite, so
    the GEMMs (and hence losses and gradients) reproduce the fixture bit for bit on any x86 host."""
    want = meta(g).get("mkl_cbwr")
    return want is None or os.environ.get("MKL_CBWR", "").split(",")[0] == want


def bit_pinned(g):
    """True when every fp32 value must match the fixture bit for bit: same MKL path AND the same
    CPU model. MKL's COMPATIBLE path alone is not enough across hosts: torch's own pointwise CPU
    kernels (the Adam update's addcdiv) round ~0.3 % of the updated parameters 1 ulp differently on
    an Intel Xeon than on the AMD EPYC the fixtures were made on (losses, gradients and both Adam
    moments still match exactly). Off the fixture's host, assert_pinned falls back to a stated fp32
    tolerance and the integer parts (RNG streams, split indices, masks, counters) stay exact."""
    want_cpu = meta(g).get("cpu")
    return same_mkl_path(g) and (want_cpu is None or want_cpu == host_cpu())


def require_pinned(g):
    """Adam-updated parameters and multi-epoch trajectories are only comparable bit for bit: the
    pre-BatchNorm bias gradients are pure rounding noise, and Adam turns any change in that noise
    into an O(lr) parameter step. Off the fixture's MKL path they are skipped."""
    if not same_mkl_path(g):
        import pytest
        pytest.skip(f"fixture pinned under MKL_CBWR={meta(g).get('mkl_cbwr')}, this run uses "
                    f"MKL_CBWR={os.environ.get('MKL_CBWR', '(default)')}")


def assert_pinned(actual, desired, g, what=""):
    """Bit-exact when bit_pinned(g); otherwise |a - d| <= 4e-6 * max|d| per tensor (≈30 ulp of the
    tensor's largest element: a different MKL path reorders every GEMM's accumulation, which moves
    the rounding of near-zero elements, e.g. the pre-BatchNorm bias gradients, by more than an ulp
    of the element itself)."""
    actual = np.asarray(actual)
    desired = np.asarray(desired)
    if bit_pinned(g) or not np.issubdtype(desired.dtype, np.floating):
        np.testing.assert_array_equal(actual, desired, err_msg=what)
        return
    scale = float(np.abs(desired).max()) if desired.size else 0.0
    np.testing.assert_allclose(actual, desired, rtol=0, atol=4e-6 * scale, err_msg=what)
