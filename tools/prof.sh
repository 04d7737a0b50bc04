#!/bin/bash
# rocprofv3 passes over a short default-shape bench: kernel stats (csv), MFMA-busy counters,
# FETCH_SIZE, WRITE_SIZE (separate --pmc passes, no tracing domains beside --kernel-trace)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-p}
B="bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-f32-line --sample-genomes 131072"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python3 $B > gpurun_out/prof_$T.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/pmc_mfma_$T -o run --output-format csv -- python3 $B > gpurun_out/pmc_mfma_$T.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_$T -o run --output-format csv -- python3 $B > gpurun_out/pmc_fetch_$T.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_$T -o run --output-format csv -- python3 $B > gpurun_out/pmc_write_$T.log 2>&1
echo "prof done rc=$?" >> gpurun_out/prof_$T.log
