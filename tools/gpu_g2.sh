cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/g2_tests.log 2>&1 || exit $?
bash tools/ab_bench.sh pk 3 ""
