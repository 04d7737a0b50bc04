# sampling-path GPU check: the sampling / decode / golden tests, the bench's sample leg, and a kernel
# trace of a 262,144-genome sample leg
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -rf -s -k "split or sampl or decode or golden or count" > gpurun_out/gpu_sel_c.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32-line --no-c5 > gpurun_out/bench_c.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-f32-line --no-c5 --sample-genomes 262144 > gpurun_out/prof_c.log 2>&1
