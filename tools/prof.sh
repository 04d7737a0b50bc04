#!/bin/bash
# rocprofv3 passes over short benches: a kernel trace + stats and an MFMA-busy counter pass over the
# C2 step only (tools/kstats.py: per-kernel time per step), then FETCH_SIZE and WRITE_SIZE passes over
# C2 + C5 + a 131,072-genome sample leg (tools/pmc.py: per-launch HBM bytes by kernel and grid).
# Each counter set is its own --pmc run; no tracing domains beside --kernel-trace.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-p}
C2="bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-f32-line --no-sample --no-c5 --no-presets --no-c1"
# (the sample leg decodes from an untrained model here: the trained-checkpoint leg's own training
# launches share the loss GEMM's grid and would mix v1 launches into the v0 medians)
ALL="bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-f32-line --no-presets --no-c1 --sample-genomes 131072 --sample-train-epochs 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python3 $C2 > gpurun_out/prof_$T.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/pmc_mfma_$T -o run --output-format csv -- python3 $C2 > gpurun_out/pmc_mfma_$T.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_$T -o run --output-format csv -- python3 $ALL > gpurun_out/pmc_fetch_$T.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_$T -o run --output-format csv -- python3 $ALL > gpurun_out/pmc_write_$T.log 2>&1
echo "prof done rc=$?" >> gpurun_out/prof_$T.log
