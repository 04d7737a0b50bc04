#!/bin/bash
# Full GPU check + default bench + a same-box A/B of env/flag variants + a kernel trace per variant:
#   bash tools/gpu_ab.sh TAG R "VAR=x|ARGS" "VAR=y|ARGS" ...   (tests skipped when TAG ends in -notest)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=$1; R=$2; shift 2
if [[ "$T" != *-notest ]]; then
  timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -rf > gpurun_out/gpu_tests_$T.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_$T.log
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 500 python3 bench.py > gpurun_out/bench_$T.log 2>&1 || exit $?
fi
bash tools/ab_bench.sh $T $R "$@" || exit $?
i=0
for v in "$@"; do
  if [[ "$v" == *"|"* ]]; then ev=${v%%|*}; args=${v#*|}; else ev=""; args=$v; fi
  env $ev timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_$i -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-f32-line --no-sample --no-c5 $args > gpurun_out/prof_${T}_$i.log 2>&1
  rc=$?; echo "prof rc=$rc" >> gpurun_out/prof_${T}_$i.log
  [ $rc -ne 0 ] && exit $rc
  i=$((i+1))
done
exit 0
