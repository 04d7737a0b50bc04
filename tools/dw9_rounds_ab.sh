# same-box A/B of the capped dW9 grid's rounds (GM2_DW9_ROUNDS) and start point
# (GM2_DW9_ROUNDS was an A/B-only knob of the round-5 build measured here; removed after: profiles/r05_dw9_rounds_ab.txt)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
bash tools/ab_bench.sh rounds 3 "X=0|" "GM2_DW9_ROUNDS=5|" "GM2_DW9_ROUNDS=6|" "GM2_DW9_ROUNDS=5 GM2_DW9_AT=0|"
