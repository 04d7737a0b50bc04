#!/bin/bash
# Round-end profile set of HEAD: a 35-step kernel trace + stats of the C2 bench with a 262,144-genome
# sample leg (per-kernel averages that agree with the live bench line), then tools/prof.sh's passes
# (C2 trace, MFMA-busy counters, FETCH_SIZE and WRITE_SIZE, each its own --pmc run).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-f}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof35_$T -o run --output-format csv -- python3 bench.py --steps 35 --warmup 5 --no-cpu-baseline --no-f32-line --no-c5 --no-presets --no-c1 --sample-genomes 262144 > gpurun_out/prof35_$T.log 2>&1 || exit $?
bash tools/prof.sh $T
