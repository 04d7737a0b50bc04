#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (each its own --pmc run) over the bench's sample leg decoding from
# the TRAINED v1 checkpoint (10 epochs, as the bench line): per-launch bytes of the sampling kernels
# on the bench's own workload (tools/pmc.py; the v1 training launches of the checkpoint share
# kernel names with the C2 step, so only the sampling kernels' rows of this summary are meaningful)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-s}
S="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-f32-line --no-c5 --no-presets --no-c1 --sample-genomes 131072"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_sfetch_$T -o run --output-format csv -- python3 $S > gpurun_out/pmc_sfetch_$T.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_swrite_$T -o run --output-format csv -- python3 $S > gpurun_out/pmc_swrite_$T.log 2>&1
echo "rc=$?" >> gpurun_out/pmc_sfetch_$T.log
