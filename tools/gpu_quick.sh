#!/bin/bash
# quick cycle: train-step / eval / gather parity tests, then a short bench
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-q}
timeout -k 10 600 python3 -m pytest tests/test_gpu_parity.py tests/test_gpu_forward.py -x -q -p no:cacheprovider -k "not test_gemm" > gpurun_out/quick_tests_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/quick_tests_$T.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-line --no-sample > gpurun_out/quick_bench_$T.log 2>&1
echo "bench rc=$?" >> gpurun_out/quick_bench_$T.log
