"""Parity at the headline configuration C2's real dimensions (BASELINE.json configs[1]): v0 preset,
G = 55,039 genes, hidden 1024, latent 64, a batch of 4096 strain rows of the synthetic F4-shaped
pan-genome matrix. One full libgm2 step (gm2_train_fwd_bwd + gm2_grad_norm) against the oracle's
explicit gradients (oracle.manual_grads_emulated: the math of the CPU oracle pinned to the
reference's goldens) evaluated on the device:

  * EXACT = fp64 (no rounding anywhere): the distance every path is measured from.
  * the reference's own arithmetic: the same math in fp32 (torch fp32 GEMMs) — for the f32 path;
    and in fp32 with the bf16 path's operand rounding (weights, post-ReLU activations, z,
    dL/dlogit, BatchNorm input gradients dY, d(mu|logvar) rounded to bf16 exactly where libgm2
    stores them) — for the bf16 path.

At this shape the gradient of the hidden layers is ill-conditioned: train-mode BatchNorm's backward
subtracts the batch mean of a mostly mean-shift signal, so ANY fp32 evaluation is up to ~5 % (max-
normalised) away from exact on those tensors while the output layers agree to ~1e-5 (measured,
printed per tensor). The bar is therefore relative to the reference arithmetic, on the norm-wise
relative error fro(a) = ||a - EXACT||_2 / ||EXACT||_2 (stable under the element-level noise of an
ill-conditioned evaluation; the max-element errors are printed next to it): per tensor,
  fro(libgm2) <= 3 * fro(reference arithmetic) + floor
(floor 2e-4 for f32, 1e-3 for bf16); losses within rel 1e-5 (f32) / 1e-4 (bf16, vs the emulated
sums), the clip norm within rel 1e-4 / 2e-2. Pre-BN Linear biases have an exactly-zero true
gradient (train-mode BatchNorm) and are compared absolutely.
"""
import numpy as np
import pytest
import torch

from gpu_helpers import perturb_bn
from oracle import vae_oracle as O

pytestmark = pytest.mark.gpu

G, H, L, B = 55039, 1024, 64, 4096
BETA = 0.1


def _prebn_bias(name):
    p = name.split(".")
    return p[0] in ("encoder", "decoder") and p[1] in ("0", "3", "6") and p[2] == "bias"


@pytest.fixture(scope="module")
def c2_state():
    from gm2.data import synthetic_pangenome
    torch.manual_seed(2024)
    P = O.init_params(G, H, L)
    S = O.init_bn_state(H)
    P, S = perturb_bn(P, S, 99)
    X = synthetic_pangenome(B, G, seed=12345)
    torch.manual_seed(5)
    eps = torch.randn(B, L)
    return P, S, X, eps


@pytest.mark.parametrize("prec", ["f32", "bf16"])
def test_c2_train_step_real_dims(prec, c2_state):
    from gm2 import native
    from gm2.data import ResidentMatrix
    from gpu_helpers import scalars, to_model
    P, S, X, eps = c2_state
    pr = native.GM2_F32 if prec == "f32" else native.GM2_BF16
    m = to_model(P, S, G, H, L, pr)
    mat = ResidentMatrix(X)
    ws = m.workspace(pr, B)
    grads = torch.zeros_like(m.params)
    loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device="cuda")
    sc = scalars(beta=BETA, wgamma=0.0, lam=0.0)
    native.train_fwd_bwd(ws, native.make_batch(mat.data, mat.ld, None, B, eps.cuda()), m.params, grads, m.bn, sc, loss)
    native.grad_norm(ws, m.params, grads, sc, loss)
    torch.cuda.synchronize()
    lt = loss.cpu().numpy()
    got = grads.cpu().numpy()
    del ws
    # fp64 references on the device
    dev = torch.device("cuda")
    Pd = {k: v.to(dev) for k, v in P.items()}
    Sd = {k: v.to(dev) for k, v in S.items()}
    x = torch.tensor(X, device=dev)
    ed = eps.to(dev)
    torch.backends.cuda.matmul.allow_tf32 = False
    exact, sums = O.manual_grads_emulated(Pd, Sd, x, ed, BETA, 0.0)
    exact = {k: v.cpu() for k, v in exact.items()}
    rnd = O.bf16_round if prec == "bf16" else None
    ref32, sums32 = O.manual_grads_emulated(Pd, Sd, x, ed, BETA, 0.0, operand_round=rnd, dtype=torch.float32)
    ref32 = {k: v.cpu().double() for k, v in ref32.items()}
    if prec == "bf16":
        sums = sums32  # the loss of the bf16 arithmetic (rounded operands)
    del x, Pd, Sd
    torch.cuda.empty_cache()
    # losses vs the reference of the same arithmetic (exact for f32, bf16-emulated for bf16)
    rtol = 1e-5 if prec == "f32" else 1e-4
    print(f"loss slots: libgm2 {lt[:3]}, reference {sums}")
    assert abs(lt[0] - sums[0]) <= rtol * abs(sums[0]), (lt[0], sums[0])
    assert abs(lt[1] - sums[1]) <= rtol * abs(sums[1]), (lt[1], sums[1])
    assert abs(lt[2] - sums[2]) <= 1e-4 * abs(sums[2]) + 1e-2, (lt[2], sums[2])
    off = m.offsets
    fails = []
    for i, (name, _) in enumerate(m.specs):
        g = got[off[i]:off[i + 1]]
        ex = exact[name].reshape(-1).numpy()
        scale = float(np.abs(ex).max()) or 1.0
        e_exact = float(np.abs(g - ex).max()) / scale
        if _prebn_bias(name):
            wscale = float(np.abs(exact[name.replace("bias", "weight")].numpy()).max())
            lim = 1e-3 if prec == "f32" else 2e-2
            if np.abs(g).max() > lim * wscale:
                fails.append(f"{name}: |g| {np.abs(g).max():.3g} vs weight scale {wscale:.3g}")
            continue
        r32 = ref32[name].reshape(-1).numpy()
        e_ref = float(np.abs(r32 - ex).max()) / scale
        nrm = float(np.linalg.norm(ex)) or 1.0
        f_gpu = float(np.linalg.norm(g - ex)) / nrm
        f_ref = float(np.linalg.norm(r32 - ex)) / nrm
        floor = 2e-4 if prec == "f32" else 1e-3
        msg = (f"{name}: libgm2 {prec} vs exact fro {f_gpu:.3g} (max-elem {e_exact:.3g}); reference arithmetic "
               f"({'fp32' if prec == 'f32' else 'fp32 + bf16 operands'}) fro {f_ref:.3g} (max-elem {e_ref:.3g})")
        ok = f_gpu <= 3 * f_ref + floor
        print(msg)
        if not ok:
            fails.append(msg)
    assert not fails, "\n".join(fails)
    # clip norm of the data gradient (no L1 in v0)
    norm = float(np.sqrt(sum((exact[n].double() ** 2).sum().item() for n in exact)))
    assert abs(lt[4] - norm) <= (1e-4 if prec == "f32" else 2e-2) * norm, (lt[4], norm)
    assert lt[3] == 0.0
