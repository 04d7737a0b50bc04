#!/bin/bash
# Round-3 GPU check: every -m gpu test, smoke(), the default bench line (incl. the C5 line), the
# 2-rank bench rehearsal through bench.py's own launcher (gloo, both ranks on the one GPU).
# Each step under its own limit; stop at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-a}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$T.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$T.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench_$T.log
[ $rc -ne 0 ] && exit $rc
GM2_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 5 --warmup 2 --no-sample --no-c5 > gpurun_out/bench2_$T.log 2>&1
rc=$?; echo "bench2 rc=$rc" >> gpurun_out/bench2_$T.log
exit $rc
