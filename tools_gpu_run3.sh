#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests9.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests9.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof9 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-sample > gpurun_out/prof9.log 2>&1
echo "prof rc=$?" >> gpurun_out/prof9.log
timeout -k 10 600 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench9.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench9.log
