"""bench-loop finiteness per configuration (diagnostic): NA waves side"""
import os
import sys
import numpy as np
import torch
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "genome-minimizer-2_amd"))
import bench  # noqa: E402
from gm2 import native  # noqa: E402
from gm2.data import ResidentMatrix, synthetic_pangenome  # noqa: E402
from gm2.model import VAE  # noqa: E402
from gm2.trainer import Adam  # noqa: E402

G, H, L, B = 55039, 1024, 64, 4096
dev = torch.device("cuda")
mat = ResidentMatrix(synthetic_pangenome(10000, G), device=dev)


def run(na, waves, nsteps=12):
    native.set_option(native.OPT_SMALL_WAVES, waves)
    torch.manual_seed(0)
    model = VAE(G, H, L, device=dev, precision=native.GM2_BF16)
    opt = Adam(model, lr=1e-3)
    ws = model.workspace(native.GM2_BF16, B)
    grads = torch.zeros_like(model.params)
    tab = bench.scalar_table(nsteps)
    tab[:, native.S_NORM_AHEAD] = na
    scal = torch.tensor(tab, dtype=torch.float32, device=dev)
    loss = torch.zeros(nsteps, native.LOSS_SLOTS, dtype=torch.float64, device=dev)
    g = torch.Generator().manual_seed(100)
    rows = torch.cat([torch.randperm(10000, generator=g)[:B] for _ in range(nsteps)]).to(torch.int32).to(dev)
    torch.cuda.manual_seed(1)
    for i in range(nsteps):
        eps = torch.randn(B, L, device=dev)
        batch = native.make_batch(mat.data, mat.ld, rows[i * B:(i + 1) * B], B, eps)
        native.train_fwd_bwd(ws, batch, model.params, grads, model.bn, scal[i], loss[i])
        native.grad_norm(ws, model.params, grads, scal[i], loss[i])
        native.adam_step(ws, model.params, grads, opt.exp_avg, opt.exp_avg_sq, scal[i])
        torch.cuda.synchronize()
    ls = loss.cpu().numpy()
    print(f"na={na} waves={waves}")
    for i in range(nsteps):
        print("  ", i, " ".join(f"{x:.6e}" for x in ls[i, :5]))
    sys.stdout.flush()


for na, w in [(0, 4), (0, 8), (1, 8)]:
    run(na, w)
