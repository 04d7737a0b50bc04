#!/bin/bash
# A5^T on the main stream: train-step parity subset, then bench x3 and a kernel trace
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-y}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2.py -k "capped_grid or c2 or train_step or staged" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/y_tests_$T.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/y_tests_$T.log
[ $rc -ne 0 ] && exit $rc
B="bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-f32-line --no-sample"
for i in 1 2 3; do timeout -k 10 200 python3 $B >> gpurun_out/y_bench_$T.log 2>&1 || exit $?; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32-line --no-sample > gpurun_out/prof_$T.log 2>&1
echo "prof rc=$?" >> gpurun_out/prof_$T.log
