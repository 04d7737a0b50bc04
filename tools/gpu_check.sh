#!/bin/bash
# One GPU check of the tree: every -m gpu test, the parity suite against the GM2_DEBUG build, the
# default bench line and a kernel trace of a short bench (tools/timeline.py reads it).
#   bash tools/gpu_check.sh TAG [skip-tests]
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-c}
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -rf > gpurun_out/gpu_tests_$T.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_$T.log
  [ $rc -ne 0 ] && exit $rc
  GM2_LIB_PATH=$PWD/genome-minimizer-2_amd/gm2/libgm2_debug.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -rf > gpurun_out/debug_parity_$T.log 2>&1
  rc=$?; echo "debug parity rc=$rc" >> gpurun_out/debug_parity_$T.log
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$T.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench_$T.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-f32-line --no-sample --no-c5 > gpurun_out/prof_$T.log 2>&1
rc=$?; echo "prof rc=$rc" >> gpurun_out/prof_$T.log
exit $rc
