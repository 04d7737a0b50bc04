"""Diagnostic (GPU): the f32 training step at the small parity shape (G 8192, H 256, L 32, B 1024,
w*gamma 0.55) with BatchNorm statistics in the GEMM epilogue vs the separate statistics pass:
per-tensor relative differences of the gradients (they should agree to fp32 rounding)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "genome-minimizer-2_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
from gm2 import native  # noqa: E402
from gm2.data import ResidentMatrix  # noqa: E402
from gpu_helpers import oracle_state, perturb_bn, scalars, synth_x, to_model  # noqa: E402
from oracle import vae_oracle as O  # noqa: E402

G, H, L, B, wg, lam = (int(a) if i < 4 else float(a) for i, a in enumerate(sys.argv[1:7])) if len(sys.argv) > 6 \
    else (8192, 256, 32, 1024, 0.55, 0.01)
P, S = perturb_bn(*oracle_state(G, H, L, G + B), seed=9)
X = synth_x(B, G, B)
torch.manual_seed(1)
eps = torch.randn(B, L)
out = {}
for epi, side in ((1, 1), (0, 1), (0, 0), (1, 0)):
    native.set_option(native.OPT_BN_EPILOGUE, epi)
    native.set_option(native.OPT_SIDE_STREAM, side)
    m = to_model(P, S, G, H, L, native.GM2_F32)
    mat = ResidentMatrix(X)
    ws = m.workspace(native.GM2_F32, B)
    grads = torch.zeros_like(m.params)
    loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device="cuda")
    native.train_fwd_bwd(ws, native.make_batch(mat.data, mat.ld, None, B, eps.cuda()), m.params, grads, m.bn,
                         scalars(beta=0.37, wgamma=wg, lam=lam), loss)
    torch.cuda.synchronize()
    out[(epi, side)] = (grads.cpu().numpy(), loss.cpu().numpy(), m.bn.cpu().numpy())
native.set_option(native.OPT_BN_EPILOGUE, 1)
native.set_option(native.OPT_SIDE_STREAM, 1)
ex, _ = O.manual_grads_emulated({k: v.cuda() for k, v in P.items()}, S, torch.tensor(X).cuda(), eps.cuda(), 0.37, wg)
keys = list(out)
print("variants (bn_epilogue, side_stream):", keys)
for k in keys:
    print(k, "loss", out[k][1][:3], "bn max diff vs first", np.abs(out[k][2] - out[keys[0]][2]).max())
for i, (n, _) in enumerate(m.specs):
    e = ex[n].reshape(-1).cpu().double().numpy()
    nrm = max(np.linalg.norm(e), 1e-30)
    print(f"{n:22s} " + "  ".join(f"{k}: {np.linalg.norm(out[k][0][m.offsets[i]:m.offsets[i + 1]] - e) / nrm:.3e}"
                                  for k in keys))
