#!/bin/bash
# all GPU tests, then in-process A/B of an option (default gemm_rem 1 0), then a short bench
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-e}
OPT=${2:-gemm_rem}
V=${3:-"1 0"}
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -rf > gpurun_out/tests_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests_$T.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/recon_ab.py $OPT $V > gpurun_out/ab_$T.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-line --no-sample > gpurun_out/bench_$T.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench_$T.log
