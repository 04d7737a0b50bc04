# same-box A/B of process-default options (GM2_OPTS="key=value,..."; gm2.h GM2_OPT_* numbers)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
bash tools/ab_bench.sh opts 3 "GM2_OPTS=|" "GM2_OPTS=6=4|" "GM2_OPTS=4=2|" "GM2_OPTS=5=0|"
