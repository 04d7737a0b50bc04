"""The reference module surface on libgm2 (model.py:100-113): `model(x)` / `forward` /
`reparameterization`, differentiable under torch autograd through gm2_backward_outputs, and the
trainer's autograd path that trains custom LossComponents (trainer.py:349-352 with_custom_loss).

Bars (exact-fp32 GEMM path): outputs rel 1e-5 vs the oracle's forward; parameter gradients rel 1e-4
of each tensor's max vs torch autograd on the oracle (pre-BN Linear biases absolute: rounding
noise); reparameterization bit-level formulas (rel 1e-6).
"""
import numpy as np
import pytest
import torch

from gpu_helpers import oracle_state, perturb_bn, rel_err, synth_x, to_model
from oracle import vae_oracle as O

pytestmark = pytest.mark.gpu

from gm2.loss_components import LossComponent

if torch.cuda.is_available():
    from gm2 import native
    from gm2.data import ResidentMatrix, StrainLoader
    from gm2.trainer import Adam, StepLR, VAETrainerBuilder

G, H, L, B = 640, 128, 16, 96


def _prebn_bias(name):
    p = name.split(".")
    return p[0] in ("encoder", "decoder") and p[1] in ("0", "3", "6") and p[2] == "bias"


def _check_grads(m, got_flat, ref, tol=1e-4, train=True):
    """Pre-BN Linear biases have an exactly-zero true gradient only under train-mode BatchNorm
    (batch mean subtraction); in eval mode BatchNorm is affine and they are compared like the rest."""
    off = m.offsets
    fails = []
    for i, (name, _) in enumerate(m.specs):
        got = got_flat[off[i]:off[i + 1]].cpu().numpy()
        r = ref[name].reshape(-1).numpy()
        if train and _prebn_bias(name):
            scale = float(np.abs(ref[name.replace("bias", "weight")].numpy()).max())
            if np.abs(got).max() > 1e-3 * scale:
                fails.append(f"{name}: |g| {np.abs(got).max():.3g} vs {scale:.3g}")
            continue
        e = rel_err(got, r)
        if e > tol:
            fails.append(f"{name}: rel err {e:.3g}")
    assert not fails, "\n".join(fails)


@pytest.mark.parametrize("train", [True, False])
def test_forward_matches_oracle(train):
    P, S = perturb_bn(*oracle_state(G, H, L, 11), seed=3)
    X = synth_x(B, G, 5)
    torch.manual_seed(4)
    eps = torch.randn(B, L)
    m = to_model(P, S, G, H, L, native.GM2_F32)
    m.train(train)
    recon, mu, lv = m(torch.tensor(X, dtype=torch.float32), eps=eps)
    S2 = {k: v.clone() for k, v in S.items()}
    r_ref, mu_ref, lv_ref = O.forward(P, S2, torch.tensor(X, dtype=torch.float32), eps, train=train)
    assert rel_err(recon.detach().cpu(), r_ref) <= 1e-5
    assert rel_err(mu.detach().cpu(), mu_ref.detach()) <= 1e-5
    assert rel_err(lv.detach().cpu(), lv_ref.detach()) <= 1e-5
    bn = m.bn.cpu().numpy()
    for i, b in enumerate(O.BNS):  # train mode updates the running statistics, eval mode does not
        np.testing.assert_allclose(bn[i, 0], S2[b + ".running_mean"].numpy(), rtol=2e-5, atol=2e-6)
        np.testing.assert_allclose(bn[i, 1], S2[b + ".running_var"].numpy(), rtol=2e-5, atol=2e-6)
    assert m.num_batches_tracked[0] == (1 if train else 0)


@pytest.mark.parametrize("train", [True, False])
def test_forward_autograd_gradients(train):
    """A loss with every output in the graph (BCE on recon, KL and a mu^2 penalty on the heads, a
    parameter term through model.parameters()) backpropagated through libgm2 == torch autograd
    through the oracle."""
    P, S = perturb_bn(*oracle_state(G, H, L, 21), seed=6)
    X = synth_x(B, G, 7)
    x = torch.tensor(X, dtype=torch.float32)
    torch.manual_seed(8)
    eps = torch.randn(B, L)
    m = to_model(P, S, G, H, L, native.GM2_F32)
    m.train(train)
    m.requires_grad_(True)

    def loss_fn(recon, mu, lv, params):
        bce = torch.nn.functional.binary_cross_entropy(recon, x.to(recon.device), reduction="sum")
        kl = -0.5 * torch.sum(1 + lv - mu.pow(2) - lv.exp())
        pen = 0.05 * torch.sum(mu ** 2) + 0.3 * recon.sum(0).abs().sum()
        reg = 1e-3 * sum(torch.sum(t ** 2) for t in params)
        return bce + 0.4 * kl + pen + reg

    recon, mu, lv = m(x, eps=eps)
    loss_fn(recon, mu, lv, m.parameters()).backward()
    got = m.params.grad.detach().clone()
    m.requires_grad_(False)
    Pl = {k: v.clone().requires_grad_(True) for k, v in P.items()}
    r2, mu2, lv2 = O.forward(Pl, {k: v.clone() for k, v in S.items()}, x, eps, train=train)
    loss_fn(r2, mu2, lv2, Pl.values()).backward()
    _check_grads(m, got, {k: v.grad for k, v in Pl.items()}, train=train)


def test_reparameterization():
    torch.manual_seed(0)
    mu = torch.randn(300, 32, device="cuda", requires_grad=True)
    lv = torch.randn(300, 32, device="cuda", requires_grad=True)
    m = to_model(*oracle_state(64, 128, 32, 0), 64, 128, 32, native.GM2_F32)
    torch.manual_seed(5)
    z = m.reparameterization(mu, lv)
    torch.manual_seed(5)
    eps = torch.randn_like(lv)
    z_ref = mu + torch.exp(0.5 * lv) * eps
    assert rel_err(z.detach().cpu(), z_ref.detach().cpu()) <= 1e-6
    w = torch.randn_like(z)
    (z * w).sum().backward()
    gmu, glv = mu.grad.clone(), lv.grad.clone()
    mu.grad = lv.grad = None
    (z_ref * w).sum().backward()
    assert rel_err(gmu.cpu(), mu.grad.cpu()) <= 1e-6
    assert rel_err(glv.cpu(), lv.grad.cpu()) <= 1e-6


class LatentPenalty(LossComponent):
    """A custom component (not one of the fused built-ins): c * sum(mu^2)."""

    def __init__(self, c=0.01):
        self.c = c

    def compute_loss(self, recon_x, data, mu, logvar, model, epoch, batch_idx):
        return self.c * torch.sum(mu ** 2)

    def get_name(self):
        return "latent_penalty"


def test_custom_loss_component_trains():
    """VAETrainerBuilder.with_custom_loss (trainer.py:349-352): the autograd path. Epoch-0 train
    losses are computed at the initial parameters of each batch; the first batch's components
    must equal the oracle's at the same parameters and noise; training must lower the loss."""
    P, S = oracle_state(G, H, L, 31)
    X = synth_x(200, G, 9)
    m = to_model(P, S, G, H, L, native.GM2_F32)
    opt = Adam(m, lr=1e-3)
    tr = (VAETrainerBuilder(m, opt, StepLR(opt, 20, 0.5)).epochs(4).gradient_clipping(1.0).print_every(100)
          .with_reconstruction_loss().with_kl_loss("linear", 0.1, 1.0).with_custom_loss(LatentPenalty(0.01))
          .build(eps_rng="cpu"))
    assert not tr.loss_tracker.fused
    mat = ResidentMatrix(X)
    torch.manual_seed(3)
    loader = StrainLoader(mat, None, 200, shuffle=False)  # one batch per epoch
    first = tr.train_epoch(loader, 0)
    # oracle at the initial parameters (same host RNG: base seed draw, then one eps draw)
    torch.manual_seed(3)
    torch.empty((), dtype=torch.int64).random_()
    eps = torch.randn(200, L)
    x = torch.tensor(X, dtype=torch.float32)
    recon, mu, lv = O.forward(P, {k: v.clone() for k, v in S.items()}, x, eps, train=True)
    bce = torch.nn.functional.binary_cross_entropy(recon, x, reduction="sum").item()
    pen = 0.01 * torch.sum(mu ** 2).item()
    assert abs(first["reconstruction"] * 200 - bce) <= 1e-5 * bce
    assert abs(first["latent_penalty"] * 200 - pen) <= 1e-4 * pen + 1e-6
    hist = [first["total"]] + [tr.train_epoch(loader, e)["total"] for e in range(1, 4)]
    assert hist[-1] < hist[0], hist
    val = tr.validate_epoch(loader, 3)
    assert np.isfinite(val["total"]) and set(val) == {"reconstruction", "kl_divergence", "latent_penalty", "total"}
