#!/bin/bash
# Generic GPU iteration: optional diagnostic script, pytest -m gpu with extra args, the default bench.
#   bash tools/gpu_run.sh TAG "PYTEST_ARGS" [DIAG_SCRIPT] [BENCH_ARGS|skip]
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=$1; PT=$2; DIAG=$3; BA=$4
if [ -n "$DIAG" ]; then
  timeout -k 10 300 python3 -u $DIAG > gpurun_out/diag_$T.log 2>&1
  rc=$?; echo "diag rc=$rc" >> gpurun_out/diag_$T.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ "$PT" != "skip" ]; then
  eval timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf "$PT" > gpurun_out/gpu_tests_$T.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_$T.log
  # assertion failures (rc 1) still let the bench run; crashes / timeouts stop here
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
fi
if [ "$BA" != "skip" ]; then
  timeout -k 10 400 python3 bench.py $BA > gpurun_out/bench_$T.log 2>&1
  rc=$?; echo "bench rc=$rc" >> gpurun_out/bench_$T.log
  [ $rc -ne 0 ] && exit $rc
fi
exit 0
