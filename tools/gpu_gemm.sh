#!/bin/bash
# GEMM microbench + one SQ counter pass over it
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
TAG=${1:-g}
timeout -k 10 300 python3 tools/gemm_bench.py 20 > gpurun_out/gemm_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "gemm_store" -d gpurun_out/pmc_gemm_$TAG -o run --output-format csv -- python3 tools/gemm_bench.py 2 > gpurun_out/pmc_gemm_$TAG.log 2>&1
echo "pmc rc=$?" >> gpurun_out/gemm_$TAG.log
