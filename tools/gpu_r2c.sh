#!/bin/bash
# new-surface GPU tests (forward/autograd/custom loss, sampling paths)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-c}
timeout -k 10 600 python3 -m pytest tests/test_gpu_forward.py tests/test_gpu_sampling.py -q -p no:cacheprovider -rA > gpurun_out/r2_new_tests_$T.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r2_new_tests_$T.log
