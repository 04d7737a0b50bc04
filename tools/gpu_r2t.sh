#!/bin/bash
# input-layer quarter launches + staging: parity tests, DDP trainer test, single-GPU A/B of the chunked launch
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-t}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ddp.py -k "quarter or staged or ddp or trainer" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/chunk_tests_$T.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/chunk_tests_$T.log
[ $rc -ne 0 ] && exit $rc
B="bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-f32-line --no-sample"
timeout -k 10 200 python3 $B --input-chunks 4 > gpurun_out/ab_c4_$T.log 2>&1 || exit $?
timeout -k 10 200 python3 $B --input-chunks 1 > gpurun_out/ab_c1_$T.log 2>&1 || exit $?
timeout -k 10 200 python3 $B --input-chunks 4 >> gpurun_out/ab_c4_$T.log 2>&1 || exit $?
timeout -k 10 200 python3 $B --input-chunks 1 >> gpurun_out/ab_c1_$T.log 2>&1
