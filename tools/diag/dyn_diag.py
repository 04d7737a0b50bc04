"""per-step losses of the libgm2 training loop at C2 dims with host-generated rows / eps (diagnostic;
compare with the CPU oracle fed the same draws)"""
import os
import sys
import torch
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "genome-minimizer-2_amd"))
from gm2 import native  # noqa: E402
from gm2.data import ResidentMatrix, synthetic_pangenome  # noqa: E402
from gm2.model import VAE  # noqa: E402
from gm2.trainer import Adam  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "tests"))
from gpu_helpers import scalars  # noqa: E402

G, H, L, B, N = [int(x) for x in sys.argv[1:6]]
prec = native.GM2_F32 if sys.argv[6] == "f32" else native.GM2_BF16
dev = torch.device("cuda")
mat = ResidentMatrix(synthetic_pangenome(10000, G), device=dev)
torch.manual_seed(0)
model = VAE(G, H, L, device=dev, precision=prec)
opt = Adam(model, lr=1e-3)
ws = model.workspace(prec, B)
grads = torch.zeros_like(model.params)
g = torch.Generator().manual_seed(100)
ge = torch.Generator().manual_seed(7)
for i in range(N):
    rows = torch.randperm(10000, generator=g)[:B].to(torch.int32).to(dev)
    eps = torch.randn(B, L, generator=ge).to(dev)
    sc = scalars(beta=0.1, step=i + 1, max_norm=1.0)
    loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device=dev)
    batch = native.make_batch(mat.data, mat.ld, rows, B, eps)
    native.train_fwd_bwd(ws, batch, model.params, grads, model.bn, sc, loss)
    native.grad_norm(ws, model.params, grads, sc, loss)
    native.adam_step(ws, model.params, grads, opt.exp_avg, opt.exp_avg_sq, sc)
    torch.cuda.synchronize()
    l = loss.cpu().numpy()
    print(i, f"recon {l[0] * -1 if l[0] < 0 else l[0]:.4e} klsum {l[2]:.4e} kl {-0.05 * l[2]:.4e} norm {l[4]:.4e}", flush=True)
