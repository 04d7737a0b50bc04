# same-box A/B of the sample leg's copy streams
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
: > gpurun_out/ab_copy.log
for r in 1 2; do
for v in 1 2 4; do
  timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-f32-line --no-c5 --copy-streams $v > gpurun_out/bench_cp.log 2>&1 || exit $?
  echo "copy-streams $v $(grep -h '"sample"' gpurun_out/bench_cp.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read())["sample"]; print(d["genomes_per_s"], d["roofline"]["launch_ms"])')" >> gpurun_out/ab_copy.log
done
done
