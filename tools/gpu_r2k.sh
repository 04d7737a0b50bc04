#!/bin/bash
# all GPU tests, a short bench and a kernel trace of the default step
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-k}
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -rf > gpurun_out/tests_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_$T.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-line --no-sample > gpurun_out/bench_$T.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-f32-line --no-sample > gpurun_out/prof_$T.log 2>&1
echo "rc=$?" >> gpurun_out/prof_$T.log
