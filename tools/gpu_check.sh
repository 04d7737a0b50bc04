#!/bin/bash
# One GPU check of HEAD: the tests selected by -k EXPR first (or none: "-"), then every -m gpu test,
# smoke(), the default bench line, and a short kernel trace of the training bench.
#   bash tools/gpu_check.sh TAG "PYTEST_K|-" [skip-bench]
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-c}; K=${2:--}
if [ "$K" != "-" ]; then
  timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -rf -k "$K" > gpurun_out/gpu_sel_$T.log 2>&1
  rc=$?; echo "pytest(sel) rc=$rc" >> gpurun_out/gpu_sel_$T.log
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -rf > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$T.log 2>&1 || exit $?
[ "$3" = "skip-bench" ] && exit 0
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$T.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-f32-line --no-sample --no-c5 --no-presets --no-c1 > gpurun_out/prof_$T.log 2>&1
rc=$?; echo "prof rc=$rc" >> gpurun_out/prof_$T.log
exit $rc
