#!/bin/bash
# one GPU iteration: GEMM parity first, then all GPU tests, GEMM microbench, short bench.
# Every step under its own time limit; stop at the first crash / timeout / GEMM failure.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
TAG=${1:-c}
timeout -k 10 400 python3 -m pytest tests/test_gpu_parity.py -k gemm -x -q -p no:cacheprovider > gpurun_out/gemm_tests_$TAG.log 2>&1
rc=$?; echo "gemm tests rc=$rc" >> gpurun_out/gemm_tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/gemm_bench.py 20 > gpurun_out/gemm_$TAG.log 2>&1
rc=$?; echo "gemm bench rc=$rc" >> gpurun_out/gemm_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench_$TAG.log
