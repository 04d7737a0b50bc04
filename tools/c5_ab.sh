cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
out=gpurun_out/ab_c5.log; : > $out
for r in 1 2; do for v in "" "--tail-split 3" "--tail-split 2" "--grid-cap 0"; do
  res=$(timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-f32-line --no-sample $v 2>/dev/null | tail -1) || exit 1
  echo "[$v] $(echo "$res" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["c5"]["ms_per_step"], d["c5"]["roofline"]["launch_ms"])')" >> $out
done; done
