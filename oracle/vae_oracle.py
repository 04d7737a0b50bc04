"""CPU oracle for the genome-minimizer-2 VAE train + sample hot path.

TEST INFRASTRUCTURE ONLY. Only `tests/`, `__graft_entry__.smoke()` and the `cpu_baseline` leg
of `bench.py` may import this module, and only as the checker / the timed CPU baseline. The
product path (`genome-minimizer-2_amd/gm2`) never imports it and fails loudly when its HIP
library is missing.

What it is: a clean-room PyTorch-CPU restatement of the reference algorithm (fp32, explicit
functional ops, same op order as the reference module so results are bit-identical at a fixed
thread count), plus an explicit (no-autograd) gradient restatement — the math the HIP kernels
implement — which the tests check against autograd.

Pinning: tests/test_oracle_golden.py checks every function here against the golden vectors in
tests/golden/*.npz, which tests/golden/make_golden.py produced by importing the reference
(/root/reference, torch 2.10 CPU, 1 thread).

Reference map (file:line in /root/reference/src/genome_minimizer_2):
  param order / init ........ training/model.py:62-93, 115-120
  encode/reparam/decode ..... training/model.py:95-113
  BCE / KL / abundance / L1 . training/training/loss_components.py:46-139, 167-202
  loss tracker .............. training/training/trainer.py:44-56
  train/val epoch ........... training/training/trainer.py:104-156
  train loop + early stop ... training/training/trainer.py:65-81, 158-189
  presets ................... utils/experiments.py:42-114, training/training/trainer.py:193-257
  sampling .................. utils/extras.py:192-203, main.py:351-370
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn.functional as F

BN_EPS = 1e-5        # nn.BatchNorm1d default
BN_MOMENTUM = 0.1    # nn.BatchNorm1d default
LINEARS = ["encoder.0", "encoder.3", "encoder.6", "mean_layer", "logvar_layer",
           "decoder.0", "decoder.3", "decoder.6", "decoder.9"]
BNS = ["encoder.1", "encoder.4", "encoder.7", "decoder.1", "decoder.4", "decoder.7"]


def param_specs(G: int, H: int, L: int):
    """(name, shape) in `model.parameters()` order (model.py:65-91)."""
    s = []
    enc_in = [G, H, H]
    for i in range(3):
        s += [(f"encoder.{3*i}.weight", (H, enc_in[i])), (f"encoder.{3*i}.bias", (H,)),
              (f"encoder.{3*i+1}.weight", (H,)), (f"encoder.{3*i+1}.bias", (H,))]
    s += [("mean_layer.weight", (L, H)), ("mean_layer.bias", (L,)),
          ("logvar_layer.weight", (L, H)), ("logvar_layer.bias", (L,))]
    dec_in = [L, H, H]
    for i in range(3):
        s += [(f"decoder.{3*i}.weight", (H, dec_in[i])), (f"decoder.{3*i}.bias", (H,)),
              (f"decoder.{3*i+1}.weight", (H,)), (f"decoder.{3*i+1}.bias", (H,))]
    s += [("decoder.9.weight", (G, H)), ("decoder.9.bias", (G,))]
    return s


def init_params(G: int, H: int, L: int):
    """Replays the reference init on the global CPU generator (model.py:62-93, 115-120):
    each nn.Linear ctor draws kaiming_uniform(a=sqrt(5)) weight + uniform bias, in construction
    order; then xavier_uniform_ on every Linear weight in modules() order and zero biases."""
    P = {}
    shapes = dict(param_specs(G, H, L))
    for lin in LINEARS:
        w = torch.empty(shapes[lin + ".weight"])
        b = torch.empty(shapes[lin + ".bias"])
        torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        fan_in = w.shape[1]
        bound = 1.0 / math.sqrt(fan_in) if fan_in > 0 else 0.0
        torch.nn.init.uniform_(b, -bound, bound)
        P[lin + ".weight"], P[lin + ".bias"] = w, b
    for bn in BNS:
        P[bn + ".weight"] = torch.ones(H)
        P[bn + ".bias"] = torch.zeros(H)
    for lin in LINEARS:
        torch.nn.init.xavier_uniform_(P[lin + ".weight"])
        P[lin + ".bias"].zero_()
    return {n: P[n] for n, _ in param_specs(G, H, L)}


def init_bn_state(H: int):
    st = {}
    for bn in BNS:
        st[bn + ".running_mean"] = torch.zeros(H)
        st[bn + ".running_var"] = torch.ones(H)
        st[bn + ".num_batches_tracked"] = torch.tensor(0, dtype=torch.long)
    return st


def flatten(P: dict) -> np.ndarray:
    return np.concatenate([v.detach().reshape(-1).numpy() for v in P.values()])


def unflatten(flat, G, H, L):
    out, o = {}, 0
    for n, shp in param_specs(G, H, L):
        k = int(np.prod(shp))
        out[n] = torch.tensor(np.asarray(flat[o:o + k], dtype=np.float32).reshape(shp))
        o += k
    return out


# ------------------------------------------------------------------------------------------
# forward (functional restatement of model.py:95-113)
# ------------------------------------------------------------------------------------------
def _bn(P, S, name, x, train):
    return F.batch_norm(x, S[name + ".running_mean"], S[name + ".running_var"],
                        P[name + ".weight"], P[name + ".bias"], training=train,
                        momentum=BN_MOMENTUM, eps=BN_EPS)


def _block(P, S, lin, bn, x, train):
    y = F.linear(x, P[lin + ".weight"], P[lin + ".bias"])
    return F.relu(_bn(P, S, bn, y, train))


def encode(P, S, x, train):
    h = x
    for i in range(3):
        h = _block(P, S, f"encoder.{3*i}", f"encoder.{3*i+1}", h, train)
    mu = F.linear(h, P["mean_layer.weight"], P["mean_layer.bias"])
    lv = F.linear(h, P["logvar_layer.weight"], P["logvar_layer.bias"])
    return mu, lv


def decode(P, S, z, train):
    h = z
    for i in range(3):
        h = _block(P, S, f"decoder.{3*i}", f"decoder.{3*i+1}", h, train)
    return torch.sigmoid(F.linear(h, P["decoder.9.weight"], P["decoder.9.bias"]))


def forward(P, S, x, eps, train):
    """(x_hat, mu, logvar); eps is the randn_like draw of model.py:102, passed explicitly."""
    mu, lv = encode(P, S, x, train)
    std = torch.exp(0.5 * lv)
    z = mu + std * eps
    return decode(P, S, z, train), mu, lv


def bump_bn_counters(S):
    for bn in BNS:
        S[bn + ".num_batches_tracked"] += 1


# ------------------------------------------------------------------------------------------
# loss components (loss_components.py) and schedules
# ------------------------------------------------------------------------------------------
def cosine_beta(t, T, lo, hi):
    """loss_components.py:187-202 (numpy float64 result)."""
    return lo + (hi - lo) / 2 * (1 + np.cos(np.pi * (t % T) / T))


@dataclass
class Preset:
    """Loss composition of create_v{0..3}_trainer (trainer.py:193-257) + experiments.py:42-114."""
    name: str
    kl_type: str
    min_beta: float
    max_beta: float
    T: int = 10
    gamma_start: float | None = None
    gamma_end: float | None = None
    weight: float = 1.0
    lambda_l1: float | None = None
    patience: int = 10
    hidden_dim: int = 512
    latent_dim: int = 32


PRESETS = {
    "v0": Preset("v0", "linear", 0.1, 1.0, hidden_dim=1024, latent_dim=64),
    "v1": Preset("v1", "linear", 0.1, 1.0, gamma_start=1.0, gamma_end=0.1, lambda_l1=0.01),
    "v2": Preset("v2", "cosine", 0.0, 1.0, T=10, gamma_start=1.0, gamma_end=0.1, lambda_l1=0.01),
    "v3": Preset("v3", "cosine", 0.1, 1.0, T=50, gamma_start=2.0, gamma_end=0.1, weight=1.0,
                 lambda_l1=0.01, patience=20),
}


@dataclass
class LossState:
    """Mutable state of the stateful components: the KL counter (loss_components.py:201-203)."""
    preset: Preset
    n_epochs: int
    counter: int = 0

    def names(self):
        n = ["reconstruction", "kl_divergence"]
        if self.preset.gamma_start is not None:
            n.append("gene_abundance")
        if self.preset.lambda_l1 is not None:
            n.append("l1_regularization")
        return n

    def beta(self, epoch):
        p = self.preset
        if p.kl_type == "linear":
            return p.min_beta + (p.max_beta - p.min_beta) * epoch / self.n_epochs
        if p.kl_type == "cosine":
            b = cosine_beta(epoch * 32 + self.counter, p.T, p.min_beta, p.max_beta)
            self.counter += 1
            return b
        return p.max_beta

    def gamma(self, epoch):
        p = self.preset
        return p.gamma_start + (p.gamma_end - p.gamma_start) * epoch / self.n_epochs


def compute_losses(ls: LossState, P, recon, x, mu, lv, epoch):
    """Components in list order, each an fp32 0-dim tensor (trainer.py:44-56); returns
    (total tensor, {name: float})."""
    parts = {}
    total = torch.tensor(0.0)
    comps = [("reconstruction", lambda: F.binary_cross_entropy(recon, x, reduction="sum"))]

    def kl():
        k = -0.5 * torch.sum(1 + lv - mu.pow(2) - lv.exp())
        return ls.beta(epoch) * k
    comps.append(("kl_divergence", kl))
    if ls.preset.gamma_start is not None:
        def ab():
            g = ls.gamma(epoch)
            return ls.preset.weight * g * torch.sum(torch.abs(recon.sum(axis=0)))
        comps.append(("gene_abundance", ab))
    if ls.preset.lambda_l1 is not None:
        def l1():
            if ls.preset.lambda_l1 == 0.0:
                return torch.tensor(0.0)
            pen = 0.0
            for v in P.values():
                pen += torch.sum(torch.abs(v))
            return ls.preset.lambda_l1 * pen
        comps.append(("l1_regularization", l1))
    for name, fn in comps:
        v = fn()
        parts[name] = v.item()
        total += v
    parts["total"] = total.item()
    return total, parts


# ------------------------------------------------------------------------------------------
# optimizer: clip_grad_norm_ (trainer.py:119) + Adam (trainer.py:120, experiments.py:260)
# ------------------------------------------------------------------------------------------
@dataclass
class AdamState:
    lr: float = 1e-3
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8
    step: int = 0
    m: dict = field(default_factory=dict)
    v: dict = field(default_factory=dict)


def clip_grads(grads: dict, max_norm: float):
    norms = [torch.linalg.vector_norm(g, 2.0) for g in grads.values()]
    total = torch.linalg.vector_norm(torch.stack(norms), 2.0)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    for g in grads.values():
        g.mul_(coef)
    return total


def adam_step(P: dict, grads: dict, st: AdamState):
    st.step += 1
    b1, b2 = st.betas
    bc1 = 1 - b1 ** st.step
    bc2 = 1 - b2 ** st.step
    step_size = st.lr / bc1
    bc2s = math.sqrt(bc2)
    with torch.no_grad():
        for n, p in P.items():
            g = grads[n]
            if n not in st.m:
                st.m[n] = torch.zeros_like(p)
                st.v[n] = torch.zeros_like(p)
            st.m[n].lerp_(g, 1 - b1)
            st.v[n].mul_(b2).addcmul_(g, g, value=1 - b2)
            denom = (st.v[n].sqrt() / bc2s).add_(st.eps)
            p.addcdiv_(st.m[n], denom, value=-step_size)


# ------------------------------------------------------------------------------------------
# one training step and whole epochs (trainer.py:104-189)
# ------------------------------------------------------------------------------------------
def train_step(P, S, ls: LossState, opt: AdamState, x, eps, epoch, max_norm=1.0):
    """zero_grad -> fwd -> losses -> backward -> clip -> Adam. Returns (parts, grads)."""
    leaves = {n: v.detach().requires_grad_(True) for n, v in P.items()}
    recon, mu, lv = forward(leaves, S, x, eps, train=True)
    bump_bn_counters(S)
    total, parts = compute_losses(ls, leaves, recon, x, mu, lv, epoch)
    total.backward()
    grads = {n: leaves[n].grad for n in P}
    clip_grads(grads, max_norm)
    for n in P:
        P[n] = leaves[n].detach()
    adam_step(P, grads, opt)
    return parts, grads


def eval_step(P, S, ls, x, eps, epoch):
    with torch.no_grad():
        recon, mu, lv = forward(P, S, x, eps, train=False)
        _, parts = compute_losses(ls, P, recon, x, mu, lv, epoch)
    return parts


def loader_perm(n):
    """RandomSampler.__iter__ on the global generator: one int64 seed, then randperm."""
    seed = int(torch.empty((), dtype=torch.int64).random_().item())
    g = torch.Generator()
    g.manual_seed(seed)
    return torch.randperm(n, generator=g)


def run_preset(P, S, preset: Preset, n_epochs, train_x, val_x, batch_size, max_norm=1.0,
               lr=1e-3, step_size=20, gamma_lr=0.5, print_every=100):
    """`v0..v3(...)` (trainer.py:261-290) with DataLoader RNG consumption replayed:
    every iterator draws a base seed; the shuffled train sampler draws its own seed."""
    ls = LossState(preset, n_epochs)
    opt = AdamState(lr=lr)
    best, bad = float("inf"), 0
    tr_hist, va_hist = [], []
    L = P["mean_layer.weight"].shape[0]
    epoch = 0
    for epoch in range(n_epochs):
        opt.lr = lr * (gamma_lr ** (epoch // step_size))
        torch.empty((), dtype=torch.int64).random_()          # _BaseDataLoaderIter base seed
        perm = loader_perm(train_x.shape[0])
        acc = {n: 0.0 for n in ls.names() + ["total"]}
        for s in range(0, train_x.shape[0], batch_size):
            xb = train_x[perm[s:s + batch_size]]
            eps = torch.randn(xb.shape[0], L)
            parts, _ = train_step(P, S, ls, opt, xb, eps, epoch, max_norm)
            for k, v in parts.items():
                acc[k] += v
        tr = {k: v / train_x.shape[0] for k, v in acc.items()}
        torch.empty((), dtype=torch.int64).random_()
        acc = {n: 0.0 for n in ls.names() + ["total"]}
        for s in range(0, val_x.shape[0], batch_size):
            xb = val_x[s:s + batch_size]
            eps = torch.randn(xb.shape[0], L)
            parts = eval_step(P, S, ls, xb, eps, epoch)
            for k, v in parts.items():
                acc[k] += v
        va = {k: v / val_x.shape[0] for k, v in acc.items()}
        tr_hist.append(tr["total"])
        va_hist.append(va["total"])
        if va["total"] < best - 1e-4:
            best, bad = va["total"], 0
        else:
            bad += 1
            if bad >= preset.patience:
                break
    return tr_hist, va_hist, epoch + 1


# ------------------------------------------------------------------------------------------
# explicit gradients: the math of the HIP kernels, checked against autograd in tests
# ------------------------------------------------------------------------------------------
def manual_grads(P, S, x, eps, beta, wgamma, lambda_l1):
    """Data + L1 gradient of total loss with explicit formulas (no autograd)."""
    f32 = torch.float32
    S = {k: v.clone() for k, v in S.items()}
    cache = []
    h = x
    B = x.shape[0]

    def blk(lin, bn, a):
        y = a @ P[lin + ".weight"].t() + P[lin + ".bias"]
        mean = y.mean(0)
        var = ((y - mean) ** 2).mean(0)
        invstd = 1.0 / torch.sqrt(var + BN_EPS)
        xhat = (y - mean) * invstd
        o = xhat * P[bn + ".weight"] + P[bn + ".bias"]
        cache.append((lin, bn, a, xhat, invstd, o))
        return torch.relu(o)
    for i in range(3):
        h = blk(f"encoder.{3*i}", f"encoder.{3*i+1}", h)
    h2 = h
    mu = h2 @ P["mean_layer.weight"].t() + P["mean_layer.bias"]
    lv = h2 @ P["logvar_layer.weight"].t() + P["logvar_layer.bias"]
    std = torch.exp(0.5 * lv)
    z = mu + std * eps
    h = z
    for i in range(3):
        h = blk(f"decoder.{3*i}", f"decoder.{3*i+1}", h)
    a5 = h
    logit = a5 @ P["decoder.9.weight"].t() + P["decoder.9.bias"]
    p = torch.sigmoid(logit)
    G = {}
    colsum = p.sum(0)
    dp = (p - x) / torch.clamp((1 - p) * p, min=1e-12) + wgamma * torch.sign(colsum)
    dl = dp * (1 - p) * p
    G["decoder.9.weight"] = dl.t() @ a5
    G["decoder.9.bias"] = dl.sum(0)
    da = dl @ P["decoder.9.weight"]

    def blk_bwd(entry, da):
        lin, bn, a, xhat, invstd, o = entry
        do = da * (o > 0).to(f32)
        sdo = do.sum(0)
        sdx = (do * xhat).sum(0)
        G[bn + ".weight"] = sdx
        G[bn + ".bias"] = sdo
        dy = P[bn + ".weight"] * invstd / B * (B * do - sdo - xhat * sdx)
        G[lin + ".weight"] = dy.t() @ a
        G[lin + ".bias"] = dy.sum(0)
        return dy @ P[lin + ".weight"]
    for e in reversed(cache[3:]):
        da = blk_bwd(e, da)
    dz = da
    dmu = dz + beta * mu
    dlv = dz * eps * std * 0.5 - 0.5 * beta * (1 - torch.exp(lv))
    G["mean_layer.weight"] = dmu.t() @ h2
    G["mean_layer.bias"] = dmu.sum(0)
    G["logvar_layer.weight"] = dlv.t() @ h2
    G["logvar_layer.bias"] = dlv.sum(0)
    da = dmu @ P["mean_layer.weight"] + dlv @ P["logvar_layer.weight"]
    for e in reversed(cache[:3]):
        da = blk_bwd(e, da)
    for n in P:
        if lambda_l1:
            G[n] = G[n] + lambda_l1 * torch.sign(P[n])
    return {n: G[n] for n in P}


def manual_grads_emulated(P, S, x, eps, beta, wgamma, operand_round=None, dtype=torch.float64):
    """manual_grads' math (the reference's autograd chain, model.py:95-113 + loss_components.py:
    49-115) evaluated in `dtype` (fp64 by default: an exact-arithmetic reference on any device),
    with `operand_round` applied to exactly the tensors libgm2's bf16 path stores as GEMM operands
    (weights, post-ReLU activations, z, dL/dlogit, every BatchNorm input gradient dY and the head
    gradient d(mu|logvar)). operand_round=None: no rounding (the exact reference for the fp32 path);
    operand_round=bf16 rounding: the bf16 path's arithmetic, so a GPU-vs-emulation difference is
    accumulation order only. Returns (grads, loss sums [BCE, sum p, KL raw])."""
    r = operand_round if operand_round is not None else (lambda t: t)
    dt = dtype
    Pd = {k: v.to(dt) for k, v in P.items()}
    Wr = {k: r(v).to(dt) if v.dim() == 2 else v.to(dt) for k, v in P.items()}
    x = x.to(dt)
    eps = eps.to(dt)
    B = x.shape[0]
    cache = []

    def blk(lin, bn, a_rounded):
        y = a_rounded @ Wr[lin + ".weight"].t() + Pd[lin + ".bias"]
        mean = y.mean(0)
        var = ((y - mean) ** 2).mean(0)
        invstd = 1.0 / torch.sqrt(var + BN_EPS)
        xhat = (y - mean) * invstd
        o = xhat * Pd[bn + ".weight"] + Pd[bn + ".bias"]
        a = torch.relu(o)
        cache.append((lin, bn, a_rounded, xhat, invstd, o))
        return r(a).to(dt)
    h = x
    for i in range(3):
        h = blk(f"encoder.{3*i}", f"encoder.{3*i+1}", h)
    h2 = h
    mu = h2 @ Wr["mean_layer.weight"].t() + Pd["mean_layer.bias"]
    lv = h2 @ Wr["logvar_layer.weight"].t() + Pd["logvar_layer.bias"]
    std = torch.exp(0.5 * lv)
    z = mu + std * eps
    h = r(z).to(dt)
    for i in range(3):
        h = blk(f"decoder.{3*i}", f"decoder.{3*i+1}", h)
    a5 = h
    logit = a5 @ Wr["decoder.9.weight"].t() + Pd["decoder.9.bias"]
    p = torch.sigmoid(logit)
    bce = -(x * torch.clamp(torch.log(p), min=-100) + (1 - x) * torch.clamp(torch.log1p(-p), min=-100)).sum()
    sums = [bce.item(), p.sum().item(), torch.sum(1 + lv - mu.pow(2) - lv.exp()).item()]
    G = {}
    dp = (p - x) / torch.clamp((1 - p) * p, min=1e-12) + wgamma
    dl = r(dp * (1 - p) * p).to(dt)
    del logit, dp
    G["decoder.9.weight"] = dl.t() @ a5
    G["decoder.9.bias"] = dl.sum(0)
    da = dl @ Wr["decoder.9.weight"]
    del dl, p

    def blk_bwd(entry, da):
        lin, bn, a, xhat, invstd, o = entry
        do = da * (o > 0).to(dt)
        sdo = do.sum(0)
        sdx = (do * xhat).sum(0)
        G[bn + ".weight"] = sdx
        G[bn + ".bias"] = sdo
        dy = Pd[bn + ".weight"] * invstd / B * (B * do - sdo - xhat * sdx)
        G[lin + ".bias"] = dy.sum(0)
        dyr = r(dy).to(dt)
        G[lin + ".weight"] = dyr.t() @ a
        return dyr @ Wr[lin + ".weight"]
    for e in reversed(cache[3:]):
        da = blk_bwd(e, da)
    dz = da
    dmu = dz + beta * mu
    dlv = dz * eps * std * 0.5 - 0.5 * beta * (1 - torch.exp(lv))
    G["mean_layer.bias"] = dmu.sum(0)
    G["logvar_layer.bias"] = dlv.sum(0)
    dmur, dlvr = r(dmu).to(dt), r(dlv).to(dt)
    G["mean_layer.weight"] = dmur.t() @ h2
    G["logvar_layer.weight"] = dlvr.t() @ h2
    da = dmur @ Wr["mean_layer.weight"] + dlvr @ Wr["logvar_layer.weight"]
    for e in reversed(cache[:3]):
        da = blk_bwd(e, da)
    return {n: G[n] for n in P}, sums


def bf16_round(t):
    """Round to bf16 (RNE) and back: what libgm2's bf16 path stores for a GEMM operand."""
    return t.to(torch.bfloat16).to(t.dtype)


# ------------------------------------------------------------------------------------------
# sampling (extras.py:192-203; main.py:351-370)
# ------------------------------------------------------------------------------------------
# sigmoid_fp32(l) > 0.5  <=>  l > 0x33C00000 (pinned by tests/golden/numerics.npz thr_*)
MASK_LOGIT_THRESHOLD = np.array([0x33C00000], dtype=np.uint32).view(np.float32)[0]


def sample_decode(P, S, z):
    with torch.no_grad():
        p = decode(P, S, z, train=False)
    return p


def decode_logits64(P, S, z):
    """fp64 logits of the last decoder layer: certifies which mask bits are rounding-sensitive."""
    P64 = {k: v.double() for k, v in P.items()}
    S64 = {k: (v.double() if v.is_floating_point() else v) for k, v in S.items()}
    with torch.no_grad():
        h = z.double()
        for i in range(3):
            h = _block(P64, S64, f"decoder.{3*i}", f"decoder.{3*i+1}", h, False)
        return F.linear(h, P64["decoder.9.weight"], P64["decoder.9.bias"])


# ------------------------------------------------------------------------------------------
# count_essential_genes (utils/extras.py:49-87): the reference's per-sample, per-gene loop
# ------------------------------------------------------------------------------------------
def count_essential_genes_loop(binary_generated_samples, essential_gene_positions):
    b = np.asarray(binary_generated_samples).astype(int)
    out = np.zeros(b.shape[0], dtype=int)
    for i in range(b.shape[0]):
        n = 0
        for _, positions in essential_gene_positions.items():
            for pos in positions:
                if pos < b.shape[1] and b[i, pos] != 0:
                    n += 1
                    break
        out[i] = n
    return out
