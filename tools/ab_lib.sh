#!/bin/bash
# same-box A/B of two library builds (release vs genome-minimizer-2_amd/gm2/libgm2_ab.so, built with
# `build_native.py --variant ab`), R alternating reps of the training-only bench, then a kernel
# trace of each:   bash tools/ab_lib.sh TAG R
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=$1; R=${2:-3}
AB=$GRAFT_REPO_ROOT/genome-minimizer-2_amd/gm2/libgm2_ab.so
bash tools/ab_bench.sh $T $R "X=0|" "GM2_LIB_PATH=$AB|" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_0 -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-f32-line --no-sample --no-c5 > gpurun_out/prof_${T}_0.log 2>&1 || exit $?
GM2_LIB_PATH=$AB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_1 -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-f32-line --no-sample --no-c5 > gpurun_out/prof_${T}_1.log 2>&1
