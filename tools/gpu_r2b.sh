#!/bin/bash
# full GPU test suite, default bench, rocprof kernel stats of a short bench
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-b}
timeout -k 10 900 python3 -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/r2_gpu_tests_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r2_gpu_tests_$T.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python3 bench.py > gpurun_out/r2_bench_$T.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/r2_bench_$T.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r2_prof_$T -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32-line > gpurun_out/r2_prof_$T.log 2>&1
echo "prof rc=$?" >> gpurun_out/r2_prof_$T.log
