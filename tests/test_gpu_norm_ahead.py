"""gm2_grad_norm with GM2_S_NORM_AHEAD: the clip statistics of the two big weight gradients
(encoder.0.weight, decoder.9.weight) taken in the epilogues of the GEMMs that write them, instead of
a second pass over 2*H*G floats (trainer.py:119 clip_grad_norm_ semantics unchanged).

The ahead path must (a) give the same total norm as the re-reading pass (a different fp64
summation order of fp32 squares: rel 1e-5), (b) actually be the one taken where both GEMMs are one
K pass -- shown by editing those gradient ranges between the calls, which the ahead statistics do
not see -- and (c) be ignored when the L1 term is present (it needs sign(theta)) or the scalar is 0.
"""
import pytest
import torch

from gm2 import native
from gm2.data import ResidentMatrix, synthetic_pangenome
from gm2.model import VAE

from gpu_helpers import scalars

pytestmark = pytest.mark.gpu


def _step(G, H, L, B, prec, seed=3):
    torch.manual_seed(seed)
    m = VAE(G, H, L, device=torch.device("cuda"), precision=prec)
    mat = ResidentMatrix(synthetic_pangenome(B + 37, G, seed=seed), device=torch.device("cuda"))
    ws = m.workspace(prec, B)
    grads = torch.zeros_like(m.params)
    eps = torch.randn(B, L, device="cuda")
    rows = torch.randperm(B + 37)[:B].to(torch.int32).cuda()
    batch = native.make_batch(mat.data, mat.ld, rows, B, eps)
    batch._keep = (mat, rows, eps)  # the Batch holds raw device pointers: keep their tensors alive
    return m, ws, grads, batch


def _norm(ws, m, grads, sc):
    loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device="cuda")
    native.grad_norm(ws, m.params, grads, sc, loss)
    torch.cuda.synchronize()
    return float(loss[4].item()), float(loss[3].item())


def _train(ws, m, grads, batch, sc):
    loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device="cuda")
    native.train_fwd_bwd(ws, batch, m.params, grads, m.bn, sc, loss)


@pytest.mark.parametrize("prec", [native.GM2_BF16, native.GM2_F32])
def test_norm_ahead_c2_shape(prec):
    G, H, L, B = 55039, 1024, 64, 4096  # the bench / C2 shape: both GEMMs are one K pass
    m, ws, grads, batch = _step(G, H, L, B, prec)
    sc0 = scalars(beta=0.1)
    sc1 = sc0.clone()
    sc1[native.S_NORM_AHEAD] = 1.0
    _train(ws, m, grads, batch, sc1)
    full, _ = _norm(ws, m, grads, sc0)
    ahead, _ = _norm(ws, m, grads, sc1)
    assert abs(ahead - full) <= 1e-5 * full, (ahead, full)
    # (b) edit both big ranges: the re-reading pass sees it, the ahead statistics do not
    off = native.param_offsets(G, H, L)
    g2 = grads.clone()
    g2[off[0]:off[1]] *= 2.0     # encoder.0.weight
    g2[off[28]:off[29]] *= 3.0   # decoder.9.weight
    edited_full, _ = _norm(ws, m, g2, sc0)
    edited_ahead, _ = _norm(ws, m, g2, sc1)
    assert edited_full > 1.5 * full
    assert abs(edited_ahead - full) <= 1e-5 * full, (edited_ahead, full)
    # (c) an L1 term: the full pass (sign(theta) and sum|theta|) whatever the scalar says
    scl0 = scalars(beta=0.1, lam=1e-4)
    scl1 = scl0.clone()
    scl1[native.S_NORM_AHEAD] = 1.0
    a = _norm(ws, m, g2, scl0)
    b = _norm(ws, m, g2, scl1)
    assert a == b and a[1] > 0


def test_norm_ahead_small_shape_matches():
    # a shape whose big GEMMs may split K: whichever path the library takes, the norm is the same
    G, H, L, B = 3001, 256, 16, 200
    m, ws, grads, batch = _step(G, H, L, B, native.GM2_BF16, seed=7)
    sc0 = scalars(beta=0.3)
    sc1 = sc0.clone()
    sc1[native.S_NORM_AHEAD] = 1.0
    _train(ws, m, grads, batch, sc1)
    full, _ = _norm(ws, m, grads, sc0)
    ahead, _ = _norm(ws, m, grads, sc1)
    assert abs(ahead - full) <= 1e-5 * full, (ahead, full)
