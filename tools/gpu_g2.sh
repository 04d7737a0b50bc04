cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "zero_copy or resident_operands or deferred or staged_next or capped_grid or quarter" > gpurun_out/g2_tests.log 2>&1 || exit $?
bash tools/ab_bench.sh zc 3 "--no-zero-copy" "" || exit $?
bash tools/trace_step.sh t11 "" && python3 tools/timeline.py t11 > gpurun_out/timeline_t11.txt
