#!/bin/bash
# parity (train step both BN routes, forward, eval, C2 real dims) -> kernel trace of a short bench
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-a}
timeout -k 10 800 python3 -m pytest tests/test_gpu_parity.py tests/test_gpu_forward.py tests/test_gpu_c2.py -x -q -p no:cacheprovider -k "not test_gemm" > gpurun_out/cyc_tests_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/cyc_tests_$T.log
[ $rc -ne 0 ] && exit $rc
bash tools/trace_step.sh $T
