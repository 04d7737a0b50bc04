#!/bin/bash
# kernel trace + stats of the sampling leg alone (bench.py with one training step)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-s}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-f32-line --no-c5 > gpurun_out/prof_$T.log 2>&1
echo "rc=$?" >> gpurun_out/prof_$T.log
