#!/bin/bash
# GEMM unit tests -> parity cycle (tests + trace) -> GEMM microbenchmark
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-a}
timeout -k 10 600 python3 -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider -k "test_gemm" > gpurun_out/gemm_tests_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gemm_tests_$T.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_cycle2.sh $T || exit $?
timeout -k 10 300 python3 tools/gemm_bench.py 10 3 > gpurun_out/gemm_bench_$T.log 2>&1
echo "rc=$?" >> gpurun_out/gemm_bench_$T.log
