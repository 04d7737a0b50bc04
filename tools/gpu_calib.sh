#!/bin/bash
# calibration: hipBLASLt on the hot GEMM shapes, libgm2's GEMM microbench, SQ counters of the
# recon / store GEMMs
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-c}
timeout -k 10 240 python3 tools/blas_ref.py > gpurun_out/blas_$T.log 2>&1 || exit $?
timeout -k 10 240 python3 tools/gemm_bench.py 20 > gpurun_out/gemm_$T.log 2>&1 || exit $?
bash tools/pmc_recon.sh $T
