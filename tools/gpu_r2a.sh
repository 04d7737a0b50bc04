#!/bin/bash
# round-2 first GPU pass: GEMM parity at the hot shapes (both main loops), then the GEMM microbench
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-a}
timeout -k 10 500 python3 -m pytest tests/test_gpu_parity.py -k "gemm" -x -q -p no:cacheprovider > gpurun_out/r2_gemm_tests_$T.log 2>&1
rc=$?; echo "gemm tests rc=$rc" >> gpurun_out/r2_gemm_tests_$T.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/gemm_bench.py 10 3 > gpurun_out/r2_gemm_bench_$T.log 2>&1
rc=$?; echo "gemm bench rc=$rc" >> gpurun_out/r2_gemm_bench_$T.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -m pytest tests/test_gpu_parity.py -k "train_step" -x -q -p no:cacheprovider > gpurun_out/r2_train_tests_$T.log 2>&1
rc=$?; echo "train tests rc=$rc" >> gpurun_out/r2_train_tests_$T.log
exit $rc
