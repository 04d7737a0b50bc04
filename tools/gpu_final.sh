#!/bin/bash
# round-end check of HEAD: every -m gpu test, smoke(), the default bench line, a kernel-trace summary,
# then the 2-rank bench rehearsal through bench.py's own launcher (gloo, both ranks on the one GPU)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${1:-z}
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -rf > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$T.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$T.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32-line --sample-genomes 262144 > gpurun_out/prof_$T.log 2>&1
rc=$?; echo "prof rc=$rc" >> gpurun_out/prof_$T.log
[ $rc -ne 0 ] && exit $rc
GM2_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 5 --warmup 2 --no-sample --no-c5 > gpurun_out/bench2_$T.log 2>&1
rc=$?; echo "bench2 rc=$rc" >> gpurun_out/bench2_$T.log
exit $rc
