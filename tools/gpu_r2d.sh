#!/bin/bash
# GEMM parity (hot shapes incl. remainder mode + odd ldc), C2 parity, then short benches:
# default, remainder off (env-free A/B needs separate processes for the side-stream priority)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-d}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -k "gemm" tests/test_gpu_c2.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -rf > gpurun_out/r2d_tests_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r2d_tests_$T.log
[ $rc -ne 0 ] && exit $rc
B="bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-line --no-sample"
timeout -k 10 200 python3 $B > gpurun_out/r2d_bench_def_$T.log 2>&1 || exit $?
GM2_SIDE_PRIO=low timeout -k 10 200 python3 $B > gpurun_out/r2d_bench_lowprio_$T.log 2>&1 || exit $?
GM2_SIDE_PRIO=high timeout -k 10 200 python3 $B > gpurun_out/r2d_bench_hiprio_$T.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/gemm_bench.py 20 > gpurun_out/r2d_gemm_$T.log 2>&1
echo "rc=$?" >> gpurun_out/r2d_gemm_$T.log
