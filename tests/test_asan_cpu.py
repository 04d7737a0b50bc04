"""SURVEY.md §5 (race detection / sanitizers): libgm2's host-side logic under AddressSanitizer.

`build_native.py --variant asan` compiles every csrc/*.hip with -DGM2_DEBUG and ASan on the host
code only (-Xarch_host -fsanitize=address: GPU sanitizers are not available on this pool) and links
tools/asan/host_asan.cpp into one executable. It needs no GPU: it sweeps the workspace layout over
7,200 (dims, precision) cases through gm2_debug_check_layout (every region 256-B aligned, disjoint,
inside the total, every named offset a region start), the resident-operand layouts and gradient
buckets, every option key against valid and invalid values (a refused value leaves the option
unchanged), the per-workspace entry points on unknown state, and the error paths of the compute
entry points. Exit 0 = all checks passed and ASan reported nothing.

The device side of the same GM2_DEBUG build (bounds checks of the gather rows, zero-copy row tables,
loss target rows, mask positions and CSR spans) runs on the GPU: tests/test_gpu_debug_build.py."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "genome-minimizer-2_amd")
EXE = os.path.join(PKG, "build_asan", "gm2_host_asan")


def _exe():
    sys.path.insert(0, PKG)
    import build_native
    try:
        return build_native.build(variant="asan")  # no-op when up to date (__graft_entry__.build() makes it)
    except RuntimeError as e:  # a diagnostic variant (best effort in build()): skip, never fail the suite
        if "fsanitize" in str(e) or "asan" in str(e).lower():
            pytest.skip(f"ASan variant not buildable on this host: {str(e)[:300]}")
        raise


def test_host_logic_under_asan():
    exe = _exe()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host_asan: all checks passed" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr


def test_asan_build_is_instrumented():
    """The driver really is an ASan build (a silently uninstrumented link would pass the test above)."""
    exe = _exe()
    with open(exe, "rb") as f:
        assert b"__asan_report_load" in f.read()
