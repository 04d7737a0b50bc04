#!/bin/bash
# round-6 GPU check: the selected tests (-k EXPR), then an optional same-box A/B of process-default
# options through tools/ab_bench.sh.   bash tools/r6_sel.sh TAG "PYTEST_K" [REPS "AB_A" "AB_B" ...]
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=$1; K=$2; shift 2
if [ "$K" != "-" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 240 --timeout-method thread -rf -k "$K" > gpurun_out/r6_sel_$T.log 2>&1
  rc=$?; echo "pytest(sel) rc=$rc" >> gpurun_out/r6_sel_$T.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ $# -gt 0 ]; then
  R=$1; shift
  bash tools/ab_bench.sh $T $R "$@" || exit $?
fi
exit 0
