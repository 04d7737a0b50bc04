#!/bin/bash
# Same-box A/B of bench.py flag sets on the C2 line and the c1_gpu (batch 64 / 32) lines.
#   bash tools/c1_ab.sh TAG R "ARGS_A" "ARGS_B" ...
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=$1; R=$2; shift 2
out=gpurun_out/c1ab_$T.log
: > $out
B="--steps 10 --warmup 3 --no-cpu-baseline --no-f32-line --no-sample --no-c5 --no-presets"
for r in $(seq 1 $R); do
  i=0
  for v in "$@"; do
    res=$(timeout -k 10 300 python3 bench.py $B $v 2>/dev/null | tail -1)
    rc=$?
    [ $rc -ne 0 ] && { echo "variant $i rc=$rc" >> $out; exit $rc; }
    echo "variant $i [$v] $(echo "$res" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["c1_gpu"]; print("C2", d["ms_per_step"], "b64", c["b64"]["ms_per_step"], "b32", c["b32"]["ms_per_step"])')" >> $out
    i=$((i+1))
  done
done
exit 0
