#!/bin/bash
# 5-stage ring for the 128x128 tiles: bit-identity tests, then bench A/B (same box)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-w}
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2.py -k "capped_grid or c2 or train_step" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/cap_tests_$T.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/cap_tests_$T.log
[ $rc -ne 0 ] && exit $rc
B="bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-f32-line --no-sample"
for i in 1 2; do
timeout -k 10 200 python3 $B --grid-cap 1 >> gpurun_out/ab_cap1_$T.log 2>&1 || exit $?
timeout -k 10 200 python3 $B --grid-cap 0 >> gpurun_out/ab_cap0_$T.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python3 $B --steps 10 --grid-cap 1 > gpurun_out/prof_$T.log 2>&1
echo "prof rc=$?" >> gpurun_out/prof_$T.log
