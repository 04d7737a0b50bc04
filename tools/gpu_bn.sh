#!/bin/bash
# BN-epilogue cycle: parity (train step both routes, forward, C2 real dims), then the option A/B
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-a}
timeout -k 10 700 python3 -m pytest tests/test_gpu_parity.py tests/test_gpu_forward.py tests/test_gpu_c2.py -x -q -p no:cacheprovider -k "not test_gemm" > gpurun_out/bn_tests_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/bn_tests_$T.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/recon_ab.py bn_epilogue 1 0 > gpurun_out/bn_ab_$T.log 2>&1
echo "ab rc=$?" >> gpurun_out/bn_ab_$T.log
