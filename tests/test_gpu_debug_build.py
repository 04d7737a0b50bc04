"""The GM2_DEBUG build (gm2/libgm2_debug.so, include/gm2_debug.h) on the GPU: its device-side
bounds checks of the index data the kernels follow stay silent on valid inputs (the smoke step and
decode, a bf16 zero-copy training step, the mask consumers) and fire on an out-of-matrix batch row
and on descending group offsets -- both chosen memory-safe (the resident operands' zero row; a loop
that never runs). Runs tests/gpu_debug_probe.py in a child process with GM2_LIB_PATH set, so this
process keeps the release library. The parity suite itself is also run once against the debug build
(profiles/r04_debug_build_parity.txt)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEBUG_LIB = os.path.join(ROOT, "genome-minimizer-2_amd", "gm2", "libgm2_debug.so")


@pytest.mark.gpu
def test_debug_build_checks():
    if not os.path.exists(DEBUG_LIB):  # (built best effort by __graft_entry__.build())
        pytest.skip("no libgm2_debug.so: build_native.py --variant debug")
    env = dict(os.environ, GM2_LIB_PATH=DEBUG_LIB)
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "gpu_debug_probe.py")], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("DEBUGPROBE ")][-1]
    f = json.loads(line[len("DEBUGPROBE "):])
    assert f["start"] == 0 and f["smoke"] == 0 and f["zero_copy"] == 0 and f["masks"] == 0, f
    assert f["loss_finite"]
    assert f["bad_row"] & 1, f     # GM2_DBG_RESIDENT_ROWS
    assert f["bad_groups"] & 8, f  # GM2_DBG_MASK_POS
