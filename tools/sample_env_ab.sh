#!/bin/bash
# sampling leg under runtime env variants: bash tools/sample_env_ab.sh TAG "VAR=x ..." "VAR=y" ...
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=$1; shift
out=gpurun_out/samp_ab_$T.log
: > $out
for v in "$@"; do
  res=$(env $v timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-f32-line --no-c5 2>/dev/null | tail -1)
  rc=$?
  [ $rc -ne 0 ] && { echo "[$v] rc=$rc" >> $out; exit $rc; }
  echo "[$v] $(echo "$res" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["sample"]; print(d["genomes_per_s"], d["roofline"]["launch_ms"])')" >> $out
done
exit 0
