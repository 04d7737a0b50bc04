#!/bin/bash
# all GPU tests, a kernel-trace profile of a short bench, GEMM phase stamps
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-i}
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -rf > gpurun_out/tests_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_$T.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32-line --no-sample > gpurun_out/prof_$T.log 2>&1 || exit $?
for s in "4096 1024 1024 1 1" "4096 1024 1024 1 0" "1024 1024 4096 0 0" "1024 55040 4096 1 0" "1024 55039 4096 1 0" "4096 1024 55040 1 1" "55040 1024 4096 1 0"; do
  timeout -k 10 60 ./tools/probe/stamp_gemm $s >> gpurun_out/stamps_$T.log 2>&1 || exit $?
done
echo done >> gpurun_out/stamps_$T.log
