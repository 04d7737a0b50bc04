#!/bin/bash
# the whole -m gpu suite against the debug build (every kernel's index checks on; tests/conftest.py
# reads the device flag words after each test and fails it on a non-zero flag)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
export GM2_LIB_PATH=$GRAFT_REPO_ROOT/genome-minimizer-2_amd/gm2/libgm2_debug.so
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > gpurun_out/gpu_debug_suite.log 2>&1
rc=$?; echo "debug suite rc=$rc" >> gpurun_out/gpu_debug_suite.log
exit $rc
