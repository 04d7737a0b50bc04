#!/bin/bash
# full round artefacts: bench (with CPU baseline + sampling), kernel-trace stats, PMC traffic passes
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
TAG=${1:-full}
timeout -k 10 900 python3 bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "recon_loss|gemm_store|adam|gemm_mask" -d gpurun_out/pmc_fetch_$TAG -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --sample-genomes 65536 > gpurun_out/pmc_fetch_$TAG.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "recon_loss|gemm_store|adam|gemm_mask" -d gpurun_out/pmc_write_$TAG -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --sample-genomes 65536 > gpurun_out/pmc_write_$TAG.log 2>&1
echo "done rc=$?" >> gpurun_out/pmc_write_$TAG.log
