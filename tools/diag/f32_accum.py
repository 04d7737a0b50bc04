"""Diagnostic (GPU): accumulation error of the exact-fp32 GEMM path on the C3 output-layer input
gradient dA5 = dL . W9 (K = G = 55,040) against fp64, next to torch's fp32 matmul and split-K
variants of gm2_gemm. Prints per-variant max / fro relative errors of dA5 and of its row-centred
version (what train-mode BatchNorm's backward keeps)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "genome-minimizer-2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from gm2 import native  # noqa: E402
from gm2.data import synthetic_pangenome  # noqa: E402
from gpu_helpers import perturb_bn  # noqa: E402
from oracle import vae_oracle as O  # noqa: E402

G, H, L, B = 55039, 512, 32, 4096
Gp = 55040
dev = torch.device("cuda")
torch.manual_seed(2024)
P = O.init_params(G, H, L)
S = O.init_bn_state(H)
P, S = perturb_bn(P, S, 99)
X = torch.tensor(synthetic_pangenome(B, G, seed=12345), device=dev, dtype=torch.float64)
W9 = P["decoder.9.weight"].to(dev).double()
b9 = P["decoder.9.bias"].to(dev).double()
# a plausible A5 (post-ReLU activations) and the v1 dL with abundance (w*gamma = 1)
g = torch.Generator(device=dev).manual_seed(3)
A5 = torch.relu(torch.randn(B, H, generator=g, device=dev, dtype=torch.float64))
p = torch.sigmoid(A5 @ W9.t() + b9)
dl = ((p - X) / torch.clamp((1 - p) * p, min=1e-12) + 1.0) * (1 - p) * p
dl32 = dl.float()
W32 = W9.float()
exact = dl32.double() @ W32.double()
centred = lambda t: t - t.mean(0, keepdim=True)  # noqa: E731
ex_c = centred(exact)


def report(name, got):
    got = got.double()
    e = (got - exact)
    ec = centred(got) - ex_c
    print(f"{name:28s} max {e.abs().max().item() / exact.abs().max().item():.3e}  "
          f"fro {e.norm().item() / exact.norm().item():.3e}  centred fro {ec.norm().item() / ex_c.norm().item():.3e}")


report("torch fp32 matmul", dl32 @ W32)
dLp = torch.zeros(B, Gp, device=dev)
dLp[:, :G] = dl32
W9p = torch.zeros(Gp, H, device=dev)
W9p[:G] = W32
for splits in (-1, 1, 4, 8, 16, 32, 64):
    C = torch.empty(B, H, device=dev)
    slab = torch.empty(max(splits, 8) * B * H + 4, device=dev)
    # dA5 = dL (K-major [B][Gp]) x W9 (MN-major [Gp][H])
    native.gemm(native.GM2_F32, dLp, Gp, W9p, H, C, H, B, H, Gp, splits, slab, True, False)
    torch.cuda.synchronize()
    report(f"gm2_gemm f32 splits={splits}", C)
