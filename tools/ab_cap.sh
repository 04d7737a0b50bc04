# same-box A/B of dW9 start points on the capped dW9 grid (GM2_OPT_GRID_CAP bit 1)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
bash tools/ab_bench.sh cap2 3 "GM2_DW9_AT=2|--grid-cap 3" "GM2_DW9_AT=3|--grid-cap 3" "GM2_DW9_AT=4|--grid-cap 3" "GM2_DW9_AT=6|--grid-cap 3" "--grid-cap 2"
