#!/bin/bash
# SQ counters of the recon-loss kernel (two --pmc passes over a short bench)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-r}
B="bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-f32-line --no-sample"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex "recon|gemm_store" --kernel-trace -d gpurun_out/pmc_sq1_$T -o run --output-format csv -- python3 $B > gpurun_out/pmc_sq1_$T.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex "recon|gemm_store" --kernel-trace -d gpurun_out/pmc_sq2_$T -o run --output-format csv -- python3 $B > gpurun_out/pmc_sq2_$T.log 2>&1
echo "rc=$?" >> gpurun_out/pmc_sq2_$T.log
