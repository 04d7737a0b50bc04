#!/bin/bash
# Same-box A/B of bench.py flag sets: runs each variant R times alternately (short training-only bench).
#   bash tools/ab_bench.sh TAG R "ARGS_A" "ARGS_B" ...     (a variant "VAR=x VAR2=y|ARGS" sets env too)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=$1; R=$2; shift 2
out=gpurun_out/ab_$T.log
: > $out
for r in $(seq 1 $R); do
  i=0
  for v in "$@"; do
    if [[ "$v" == *"|"* ]]; then ev=${v%%|*}; args=${v#*|}; else ev=""; args=$v; fi
    res=$(env $ev timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-f32-line --no-sample --no-c5 --no-presets --no-c1 $args 2>/dev/null | tail -1)
    rc=$?
    [ $rc -ne 0 ] && { echo "variant $i rc=$rc" >> $out; exit $rc; }
    echo "variant $i [$v] $(echo "$res" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["launch_ms"])')" >> $out
    i=$((i+1))
  done
done
exit 0
