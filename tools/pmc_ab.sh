#!/bin/bash
# PMC passes (WRITE_SIZE, FETCH_SIZE, SQ busy/wait/MFMA) of kernels matching REGEX for each bench flag
# set:  bash tools/pmc_ab.sh TAG REGEX "ARGS_A" "ARGS_B" ...
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=$1; RX=$2; shift 2
B="bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-f32-line --no-sample --no-c5"
i=0
for v in "$@"; do
  for pass in "WRITE_SIZE" "FETCH_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"; do
    n=$(echo $pass | cut -d' ' -f1)
    timeout -k 10 120 rocprofv3 --pmc $pass --kernel-include-regex "$RX" --kernel-trace -d gpurun_out/pmc_${T}_${i}_$n -o run --output-format csv -- python3 $B $v > gpurun_out/pmc_${T}_${i}_$n.log 2>&1 || exit $?
  done
  i=$((i+1))
done
exit 0
