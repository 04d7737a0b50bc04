#!/bin/bash
# Adam non-temporal A/B (kernel trace of short benches) + GEMM phase stamps for the hot shapes
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-h}
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32-line --no-sample"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/adnt1_$T -o run --output-format csv -- python3 $B > gpurun_out/adnt1_$T.log 2>&1 || exit $?
GM2_ADAM_NT=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/adnt0_$T -o run --output-format csv -- python3 $B > gpurun_out/adnt0_$T.log 2>&1 || exit $?
for s in "4096 1024 1024 1 1" "4096 1024 1024 1 0" "1024 1024 4096 0 0" "1024 55040 4096 1 0" "1024 55039 4096 1 0" "4096 1024 55040 1 1"; do
  timeout -k 10 60 ./tools/probe/stamp_gemm $s >> gpurun_out/stamps_$T.log 2>&1 || exit $?
done
echo done >> gpurun_out/stamps_$T.log
