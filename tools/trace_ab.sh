#!/bin/bash
# kernel-trace A/B of two library builds: bash tools/trace_ab.sh TAG R "ENV_A" "ENV_B" (alternating,
# 20-step C2 benches under rocprofv3 --kernel-trace; summarise with tools/trace_ab.py TAG)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=$1; R=$2; shift 2
for r in $(seq 1 $R); do
  i=0
  for v in "$@"; do
    env $v timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tab_${T}_${i}_${r} -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-line --no-sample --no-c5 > gpurun_out/tab_${T}_${i}_${r}.log 2>&1 || exit $?
    i=$((i+1))
  done
done
exit 0
