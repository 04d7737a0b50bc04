#!/bin/bash
# Same-box A/B of process environments (A/B switches read by libgm2) on the C2 line and the c1_gpu lines.
#   bash tools/c1_env_ab.sh TAG R "VAR=x" "VAR=y" ...     ("-" = no variable)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=$1; R=$2; shift 2
out=gpurun_out/c1env_$T.log
: > $out
B="--steps 10 --warmup 3 --no-cpu-baseline --no-f32-line --no-sample --no-c5"
for r in $(seq 1 $R); do
  for v in "$@"; do
    if [ "$v" = "-" ]; then ev=""; else ev=$v; fi
    res=$(env $ev timeout -k 10 300 python3 bench.py $B 2>/dev/null | tail -1)
    rc=$?
    [ $rc -ne 0 ] && { echo "[$v] rc=$rc" >> $out; exit $rc; }
    echo "[$v] $(echo "$res" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["c1_gpu"]; p=d["presets"]; print("C2", d["ms_per_step"], "b64", c["b64"]["ms_per_step"], "b32", c["b32"]["ms_per_step"], "v1", p["v1"]["ms_per_step"])')" >> $out
  done
done
exit 0
