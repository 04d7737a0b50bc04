cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
bash tools/ab_bench.sh fence 2 "GM2_EVENT_FENCE=system|--defer-adam 1" "--defer-adam 1" "--defer-adam 1 --dw9-last 1" || exit $?
bash tools/trace_step.sh t8 "--defer-adam 1" && python3 tools/timeline.py t8 > gpurun_out/timeline_t8.txt
