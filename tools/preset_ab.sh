#!/bin/bash
# Same-box A/B of bench.py flag sets on the C2 line and the v1 / v2 / v3 preset lines.
#   bash tools/preset_ab.sh TAG R "ARGS_A" "ARGS_B" ...
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=$1; R=$2; shift 2
out=gpurun_out/presetab_$T.log
: > $out
B="--steps 10 --warmup 3 --no-cpu-baseline --no-f32-line --no-sample --no-c5 --no-c1"
for r in $(seq 1 $R); do
  i=0
  for v in "$@"; do
    res=$(timeout -k 10 300 python3 bench.py $B $v 2>/dev/null | tail -1)
    rc=$?
    [ $rc -ne 0 ] && { echo "variant $i rc=$rc" >> $out; exit $rc; }
    echo "variant $i [$v] $(echo "$res" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["presets"]; print("C2", d["ms_per_step"], d["roofline"]["launch_ms"], " ".join(k + " " + str(p[k]["ms_per_step"]) + " " + str(p[k]["roofline"]["launch_ms"]) for k in ("v1", "v2", "v3")))')" >> $out
    i=$((i+1))
  done
done
exit 0
