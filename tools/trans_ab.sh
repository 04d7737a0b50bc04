# same-box A/B: dW9's transposed store from registers (GM2_TRANS_DIRECT=1, EPI 2) vs through LDS (EPI 3)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
bash tools/ab_bench.sh trans 3 "X=0|" "GM2_TRANS_DIRECT=1|"
