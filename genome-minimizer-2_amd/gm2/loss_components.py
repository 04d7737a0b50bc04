"""Loss components — mirror of src/genome_minimizer_2/training/training/loss_components.py.

The reference's plugin API (LossComponent ABC, compute_loss(recon_x, data, mu, logvar, model,
epoch, batch_idx), get_name) is kept with the reference's compute_loss formulas (torch ops on
whatever device the tensors live). Two ways a component is trained (gm2/trainer.py):
  * fused (the built-ins, each at most once, reconstruction included — every v0..v3 preset): the
    component contributes its schedule scalar to the HIP kernels (the BCE/abundance epilogue of the
    output GEMM, the KL in the reparameterization kernel, L1 in the optimizer pass) and turns the
    kernels' raw device sums back into the reference's per-batch fp32 values (scalars / value);
  * autograd (any other combination, e.g. a custom component added with with_custom_loss): every
    component's compute_loss runs on the outputs of model(x) — libgm2's forward — and torch
    autograd hands the gradients back to libgm2's backward (VAE.forward, gm2_backward_outputs).
    Documented as the non-fused path: the loss math of the components is torch, the model is HIP.

Schedules are the reference formulas verbatim in semantics (same float64 host arithmetic), and the
KL counter is stateful exactly as loss_components.py:199-203 (advances on train AND val calls).
"""
from __future__ import annotations

from abc import ABC, abstractmethod

import numpy as np
import torch


class LossComponent(ABC):
    """loss_components.py:16-43."""

    @abstractmethod
    def compute_loss(self, recon_x, data, mu, logvar, model, epoch, batch_idx):
        """The loss tensor of this component (differentiable: torch autograd)."""

    @abstractmethod
    def get_name(self) -> str: ...

    # fused-path hooks -------------------------------------------------------------------------
    def scalars(self, epoch: int) -> dict:
        """Per-batch scalars for the kernels ({'beta'|'wgamma'|'lambda': float})."""
        return {}

    def value(self, raw: np.ndarray, sc: dict) -> np.float32:
        """The reference's per-batch fp32 loss from the kernel sums `raw` (gm2.h loss record)."""
        raise NotImplementedError


class ReconstructionLoss(LossComponent):
    """BCE(recon_x, data, reduction='sum') (loss_components.py:46-53)."""

    def compute_loss(self, recon_x, data, mu, logvar, model, epoch, batch_idx):
        return torch.nn.functional.binary_cross_entropy(recon_x, data, reduction="sum")

    def get_name(self):
        return "reconstruction"

    def value(self, raw, sc):
        return np.float32(raw[0])


def cosine_annealing_schedule(t, T, min_beta, max_beta):
    """loss_components.py:187-202."""
    return min_beta + (max_beta - min_beta) / 2 * (1 + np.cos(np.pi * (t % T) / T))


class KLDivergenceLoss(LossComponent):
    """beta * (-0.5 * sum(1 + lv - mu^2 - exp(lv))) with linear / cosine / constant beta
    (loss_components.py:56-91)."""

    def __init__(self, scheduler_type="linear", min_beta=0.0, max_beta=1.0, T=10):
        self.scheduler_type = scheduler_type
        self.min_beta = min_beta
        self.max_beta = max_beta
        self.T = T
        self.counter = 0
        self.n_epochs = 1000  # updated by VAETrainer.setup_loss_components (trainer.py:99-102)

    def compute_loss(self, recon_x, data, mu, logvar, model, epoch, batch_idx):
        kl_loss = -0.5 * torch.sum(1 + logvar - mu.pow(2) - logvar.exp())
        return self.beta(epoch) * kl_loss

    def get_name(self):
        return "kl_divergence"

    def beta(self, epoch):
        if self.scheduler_type == "linear":
            return self.min_beta + (self.max_beta - self.min_beta) * epoch / self.n_epochs
        if self.scheduler_type == "cosine":
            t = epoch * 32 + self.counter
            b = cosine_annealing_schedule(t, self.T, self.min_beta, self.max_beta)
            self.counter += 1
            return b
        return self.max_beta

    def scalars(self, epoch):
        return {"beta": self.beta(epoch)}

    def value(self, raw, sc):
        kl = np.float32(-0.5) * np.float32(raw[2])
        return np.float32(np.float32(sc["beta"]) * kl)


class GeneAbundanceLoss(LossComponent):
    """weight * gamma * sum_g |sum_b p_bg| with linear gamma (loss_components.py:94-118)."""

    def __init__(self, gamma_start=0.0, gamma_end=1.0, weight=1.0):
        self.gamma_start = gamma_start
        self.gamma_end = gamma_end
        self.weight = weight
        self.n_epochs = 1000

    def gamma(self, epoch):
        return self.gamma_start + (self.gamma_end - self.gamma_start) * epoch / self.n_epochs

    def compute_loss(self, recon_x, data, mu, logvar, model, epoch, batch_idx):
        total_gene_number = recon_x.sum(axis=0)
        return self.weight * self.gamma(epoch) * torch.sum(torch.abs(total_gene_number))

    def get_name(self):
        return "gene_abundance"

    def scalars(self, epoch):
        return {"wgamma": self.weight * self.gamma(epoch)}

    def value(self, raw, sc):
        return np.float32(np.float32(sc["wgamma"]) * np.float32(raw[1]))


class L1RegularizationLoss(LossComponent):
    """lambda * sum over ALL parameters of |theta| (loss_components.py:121-139, 167-184)."""

    def __init__(self, lambda_l1=0.0):
        self.lambda_l1 = lambda_l1

    def compute_loss(self, recon_x, data, mu, logvar, model, epoch, batch_idx):
        if self.lambda_l1 == 0.0:
            return torch.tensor(0.0, device=recon_x.device)
        return l1_regularization(model, self.lambda_l1)

    def get_name(self):
        return "l1_regularization"

    def scalars(self, epoch):
        return {"lambda": self.lambda_l1}

    def value(self, raw, sc):
        if self.lambda_l1 == 0.0:
            return np.float32(0.0)
        return np.float32(np.float32(self.lambda_l1) * np.float32(raw[3]))


class L2RegularizationLoss(LossComponent):
    """Declared by the reference (loss_components.py:142-164) but used by no trainer preset; trains
    on the autograd path."""

    def __init__(self, lambda_l2: float = 0.01):
        self.lambda_l2 = lambda_l2

    def compute_loss(self, recon_x, data, mu, logvar, model, epoch, batch_idx):
        if self.lambda_l2 == 0.0:
            return torch.tensor(0.0, device=recon_x.device)
        l2_penalty = 0
        for param in model.parameters():
            l2_penalty += torch.sum(param ** 2)
        return self.lambda_l2 * l2_penalty

    def get_name(self):
        return "l2_regularization"


def l1_regularization(model, lambda_l1):
    """loss_components.py:167-184: lambda * sum over model.parameters() of sum|theta|."""
    l1_penalty = 0.0
    for param in model.parameters():
        l1_penalty += torch.sum(torch.abs(param))
    return lambda_l1 * l1_penalty


BUILTIN = (ReconstructionLoss, KLDivergenceLoss, GeneAbundanceLoss, L1RegularizationLoss)



def fused_supported(components):
    """The fused HIP path evaluates each built-in at most once and always the reconstruction term."""
    types = [type(c) for c in components]
    return (all(t in BUILTIN for t in types) and len(set(types)) == len(types)
            and ReconstructionLoss in types)


__all__ = ["LossComponent", "ReconstructionLoss", "KLDivergenceLoss", "GeneAbundanceLoss",
           "L1RegularizationLoss", "L2RegularizationLoss", "l1_regularization", "cosine_annealing_schedule",
           "fused_supported"]
