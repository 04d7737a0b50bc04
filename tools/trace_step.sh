#!/bin/bash
# kernel trace of a short default bench (one rocprofv3 pass, csv); extra env (e.g. GM2_SIDE_STREAM=0)
# is inherited from the caller
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-t}; X=$2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-f32-line --no-sample --no-c5 --no-presets --no-c1 $X > gpurun_out/prof_$T.log 2>&1
echo "rc=$?" >> gpurun_out/prof_$T.log
