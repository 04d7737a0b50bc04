#!/bin/bash
# GEMM + C2 parity, stamps of the odd-ldc input-layer gradient shape, short bench
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-j}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -rf > gpurun_out/tests_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_$T.log
[ $rc -ne 0 ] && exit $rc
for s in "1024 55040 4096 1 0" "1024 55039 4096 1 0"; do
  timeout -k 10 60 ./tools/probe/stamp_gemm $s >> gpurun_out/stamps_$T.log 2>&1 || exit $?
done
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-line --no-sample > gpurun_out/bench_$T.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench_$T.log
