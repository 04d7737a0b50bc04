# sampling tests + same-box A/B of the single-product tier's gate (GM2_SINGLE_BOUND) and the tier off
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -rf -k "split or sampl or decode or golden or count" > gpurun_out/gpu_sel_sb.log 2>&1 || exit $?
: > gpurun_out/ab_sb.log
for v in "GM2_SINGLE_BOUND=0.25" "GM2_SINGLE_BOUND=0.1" "GM2_SINGLE_BOUND=0.05" "GM2_SINGLE_BOUND=0"; do
  env $v timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-f32-line --no-c5 > gpurun_out/bench_sb.log 2>&1 || exit $?
  echo "$v $(grep -h '"sample"' gpurun_out/bench_sb.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read())["sample"]; print(d["genomes_per_s"], d["single_tiles"], d["split_tiles"], d["exact_tiles"], d["band_elements"], d["roofline"]["launch_ms"])')" >> gpurun_out/ab_sb.log
done
