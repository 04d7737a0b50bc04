#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -k "train_step or eval_forward" -s > gpurun_out/gpu_tests2.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke2.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/smoke2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-sample > gpurun_out/prof1.log 2>&1
echo "prof rc=$?" >> gpurun_out/prof1.log
