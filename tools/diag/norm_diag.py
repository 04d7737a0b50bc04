"""per-tensor gradient norms of one training call (diagnostic)"""
import os
import sys
import torch
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, os.path.join(ROOT, "genome-minimizer-2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
from gm2 import native  # noqa: E402
from gm2.data import ResidentMatrix, synthetic_pangenome  # noqa: E402
from gm2.model import VAE  # noqa: E402
from gpu_helpers import scalars  # noqa: E402

G, H, L, B = [int(x) for x in sys.argv[1:5]]
prec = int(sys.argv[5])
use_rows = int(sys.argv[6])
torch.manual_seed(3)
m = VAE(G, H, L, device=torch.device("cuda"), precision=prec)
mat = ResidentMatrix(synthetic_pangenome(B + 37, G, seed=3), device=torch.device("cuda"))
ws = m.workspace(prec, B)
grads = torch.zeros_like(m.params)
eps = torch.randn(B, L, device="cuda")
rows = torch.randperm(B + 37)[:B].to(torch.int32).cuda() if use_rows else None
batch = native.make_batch(mat.data, mat.ld, rows, B, eps)
sc = scalars(beta=0.1)
loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device="cuda")
native.train_fwd_bwd(ws, batch, m.params, grads, m.bn, sc, loss)
native.grad_norm(ws, m.params, grads, sc, loss)
torch.cuda.synchronize()
print("loss", loss.cpu().numpy()[:5])
off = native.param_offsets(G, H, L)
for i in range(30):
    gsl = grads[off[i]:off[i + 1]].double()
    print(i, off[i + 1] - off[i], f"{gsl.norm().item():.4e}", f"{gsl.abs().max().item():.4e}", bool(torch.isfinite(gsl).all()))
