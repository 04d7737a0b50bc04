#!/bin/bash
# DDP gradient exchange tests (2 ranks over gloo on the one GPU)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-u}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ddp.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ddp_tests_$T.log 2>&1
echo "tests rc=$?" >> gpurun_out/ddp_tests_$T.log
