#!/bin/bash
# GPU tests (selected by -k EXPR, or all with "all"), an A/B of bench flag sets, and kernel traces of
# the listed variants:  bash tools/gpu_ab_trace.sh TAG "PYTEST_K|all|skip" R "ARGS_A" "ARGS_B" ...
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=$1; K=$2; R=$3; shift 3
if [ "$K" != "skip" ]; then
  if [ "$K" = "all" ]; then sel=(); else sel=(-k "$K"); fi
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -rf "${sel[@]}" > gpurun_out/gpu_tests_$T.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_$T.log
  [ $rc -ne 0 ] && exit $rc
fi
bash tools/ab_bench.sh $T $R "$@" || exit $?
i=0
for v in "$@"; do
  if [[ "$v" == *"|"* ]]; then ev=${v%%|*}; args=${v#*|}; else ev=""; args=$v; fi
  env $ev timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_$i -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-f32-line --no-sample --no-c5 --no-presets --no-c1 $args > gpurun_out/prof_${T}_$i.log 2>&1
  rc=$?; echo "prof rc=$rc" >> gpurun_out/prof_${T}_$i.log
  [ $rc -ne 0 ] && exit $rc
  i=$((i+1))
done
exit 0
