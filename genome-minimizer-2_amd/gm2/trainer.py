"""Training engine — mirror of src/genome_minimizer_2/training/training/trainer.py on libgm2.

Same public surface: TrainingConfig, LossTracker, EarlyStopping, VAETrainer (setup_loss_components,
train_epoch, validate_epoch, train), create_v{0..3}_trainer, v0..v3, VAETrainerBuilder; same
return values ((train_totals, val_totals, epochs_run)), same stdout lines, same early-stopping and
StepLR semantics. What changes is the per-batch body (trainer.py:109-124): one fused forward +
backward launch sequence, the clip statistics and one fused L1+clip+Adam pass, all on the GPU,
with the per-component batch losses kept on the device and read ONCE per epoch (the reference
syncs with .item() per component per batch, trainer.py:52-55).

Data parallel (gm2/ddp.py): with torch.distributed initialised (one process per GPU,
RCCL), each rank runs its contiguous slice of every global batch; the gradient buffer is
SUM-all-reduced in buckets overlapped with the backward, before the clip statistics; the L1 term
and the clip are applied once, after the reduction, identically on every rank. BatchNorm batch
statistics are per rank (standard DDP); running statistics are averaged over ranks every epoch.
"""
from __future__ import annotations

import os

import math
from dataclasses import dataclass
from typing import Dict, List, Tuple

import numpy as np
import torch

from . import native
from .data import StrainLoader, as_strain_loader
from .ddp import (GradSync, average_running_stats, enable_sync_bn, get_dist, rank_share, rank_slice, rank_world,
                  train_rows_cap,
                  reduce_loss_rows)
from .loss_components import (GeneAbundanceLoss, KLDivergenceLoss, L1RegularizationLoss, LossComponent,
                              ReconstructionLoss, fused_supported)


@dataclass
class TrainingConfig:
    """trainer.py:23-31."""
    n_epochs: int
    max_norm: float
    lambda_l1: float = 0.0
    patience: int = 10
    min_delta: float = 1e-4
    print_every: int = 100


class Adam:
    """torch.optim.Adam(model.parameters(), lr) equivalent over the flat parameter buffer
    (experiments.py:260): betas (0.9, 0.999), eps 1e-8, no weight decay. State lives in two flat
    fp32 device buffers; the update runs in libgm2's fused L1+clip+Adam kernel."""

    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        self.model = model
        self.param_groups = [{"lr": lr, "initial_lr": lr}]
        self.defaults = {"lr": lr, "betas": betas, "eps": eps}
        self.betas, self.eps = betas, eps
        self.step_count = 0
        self.exp_avg = torch.zeros_like(model.params)
        self.exp_avg_sq = torch.zeros_like(model.params)

    def zero_grad(self, set_to_none=True):
        pass  # gradients are overwritten by every fused backward

    def state_dict(self):
        return {"step": self.step_count, "lr": self.param_groups[0]["lr"], "exp_avg": self.exp_avg.cpu(),
                "exp_avg_sq": self.exp_avg_sq.cpu()}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        self.param_groups[0]["lr"] = float(sd["lr"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])


class StepLR:
    """torch.optim.lr_scheduler.StepLR(step_size, gamma) (experiments.py:261-265)."""

    def __init__(self, optimizer, step_size=20, gamma=0.5):
        self.optimizer, self.step_size, self.gamma = optimizer, step_size, gamma
        self.base_lr = optimizer.param_groups[0]["lr"]
        self.last_epoch = 0

    def step(self):
        self.last_epoch += 1
        self.optimizer.param_groups[0]["lr"] = self.base_lr * self.gamma ** (self.last_epoch // self.step_size)

    def get_last_lr(self):
        return [self.optimizer.param_groups[0]["lr"]]


def _dist_world():
    return rank_world()[1]


class LossTracker:
    """trainer.py:34-62 (per-epoch lists of epoch-averaged component losses)."""

    def __init__(self, loss_components: List[LossComponent]):
        self.loss_components = loss_components
        self.fused = fused_supported(loss_components)
        self.train_losses = {c.get_name(): [] for c in loss_components}
        self.val_losses = {c.get_name(): [] for c in loss_components}
        self.train_losses["total"] = []
        self.val_losses["total"] = []

    def batch_scalars(self, epoch):
        """Run every component's schedule once for this batch, in list order (the KL counter
        advances exactly as in compute_total_loss)."""
        sc = {"beta": 0.0, "wgamma": 0.0, "lambda": 0.0}
        per = []
        for c in self.loss_components:
            s = c.scalars(epoch)
            sc.update(s)
            per.append(s)
        return sc, per

    def batch_values(self, raw, per):
        """Reference per-batch floats: each component's fp32 value, and their fp32 sum in list order
        (total = tensor(0.) += loss ..., trainer.py:48-55)."""
        out = {}
        total = np.float32(0.0)
        for c, s in zip(self.loss_components, per):
            v = c.value(raw, s)
            out[c.get_name()] = float(v)
            total = np.float32(total + v)
        out["total"] = float(total)
        return out

    def compute_total_loss(self, recon_x, data, mu, logvar, model, epoch, batch_idx, is_training=True):
        """trainer.py:44-56 (the autograd path): components in list order, each .item()'d."""
        individual = {}
        total = torch.tensor(0.0, device=recon_x.device)
        for c in self.loss_components:
            loss = c.compute_loss(recon_x, data, mu, logvar, model, epoch, batch_idx)
            individual[c.get_name()] = loss.item()
            total += loss
        individual["total"] = total.item()
        return total, individual

    def update_epoch_losses(self, epoch_losses: Dict[str, float], is_training=True):
        d = self.train_losses if is_training else self.val_losses
        for name, v in epoch_losses.items():
            d[name].append(v)


class EarlyStopping:
    """trainer.py:65-81."""

    def __init__(self, patience=10, min_delta=1e-4):
        self.patience = patience
        self.min_delta = min_delta
        self.best_loss = float("inf")
        self.epochs_no_improve = 0

    def should_stop(self, val_loss: float) -> bool:
        if val_loss < self.best_loss - self.min_delta:
            self.best_loss = val_loss
            self.epochs_no_improve = 0
            return False
        self.epochs_no_improve += 1
        return self.epochs_no_improve >= self.patience


class VAETrainer:
    """trainer.py:84-189 on libgm2. `eps_rng`: 'device' draws the reparameterization noise with
    torch's generator on the model's device (what the reference does on a GPU: randn_like on a
    cuda tensor); 'cpu' draws it from the global CPU generator (what the reference does on CPU;
    used by the parity tests against the CPU oracle). `sync_bn` (data parallel only; default from
    env GM2_SYNC_BN): train-mode BatchNorm over the global batch (gm2.ddp.enable_sync_bn)."""

    def __init__(self, model, optimizer, scheduler, config: TrainingConfig, eps_rng="device", sync_bn=None):
        self.model = model
        self.optimizer = optimizer
        self.scheduler = scheduler
        self.config = config
        self.loss_tracker = None
        self.early_stopping = EarlyStopping(config.patience, config.min_delta)
        self.eps_rng = eps_rng
        self.device = model.device
        self.scal = torch.zeros(native.NUM_SCALARS, dtype=torch.float32, device=self.device)
        self.grads = torch.zeros_like(model.params)
        self.last_grad_norm = None
        self._sync = None
        self.sync_bn = bool(int(os.environ.get("GM2_SYNC_BN", "0"))) if sync_bn is None else bool(sync_bn)

    def setup_loss_components(self, loss_components: List[LossComponent]):
        self.loss_tracker = LossTracker(loss_components)
        for c in loss_components:
            if hasattr(c, "n_epochs"):
                c.n_epochs = self.config.n_epochs

    # ------------------------------------------------------------------------------ helpers
    def _eps(self, n):
        L = self.model.latent_dim
        if self.eps_rng == "cpu":
            return torch.randn(n, L).to(self.device)
        return torch.randn(n, L, device=self.device)

    def _scalar_row(self, sc, adam_step=None, norm_ahead=False):
        v = np.zeros(native.NUM_SCALARS, dtype=np.float64)
        # single process, fused step: grads go from gm2_train_fwd_bwd to gm2_grad_norm untouched
        v[native.S_NORM_AHEAD] = 1.0 if norm_ahead else 0.0
        v[native.S_BETA] = sc["beta"]
        v[native.S_WGAMMA] = sc["wgamma"]
        v[native.S_LAMBDA] = sc["lambda"]
        v[native.S_MAX_NORM] = self.config.max_norm if self.config.max_norm is not None else 0.0
        opt = self.optimizer
        b1, b2 = opt.betas
        if adam_step is not None:
            lr = opt.param_groups[0]["lr"]
            v[native.S_NEG_STEP] = -(lr / (1 - b1 ** adam_step))
            v[native.S_BC2_SQRT] = math.sqrt(1 - b2 ** adam_step)
        v[native.S_ONE_MINUS_B1] = 1 - b1
        v[native.S_BETA2] = b2
        v[native.S_ONE_MINUS_B2] = 1 - b2
        v[native.S_ADAM_EPS] = opt.eps
        return v.astype(np.float32)

    def _upload(self, rows_np):
        """One H2D copy of the epoch's per-batch scalar table (no per-batch host sync)."""
        t = torch.from_numpy(np.stack(rows_np) if rows_np else np.zeros((1, native.NUM_SCALARS), np.float32))
        return t.to(self.device)

    def _bump_bn(self):
        self.model.num_batches_tracked = [n + 1 for n in self.model.num_batches_tracked]

    def _grad_sync(self, dist):
        if self._sync is None or self._sync.dist is not dist:
            # GM2_GRAD_EXCHANGE=bf16 (main.py --grad-exchange): the big weight buckets in bf16
            self._sync = GradSync(dist, self.model, self.grads, exchange=os.environ.get("GM2_GRAD_EXCHANGE", "f32"))
        return self._sync

    def _epoch_values(self, raw, pers, n_rows):
        epoch_losses = None
        for bi, per in enumerate(pers):
            vals = self.loss_tracker.batch_values(raw[bi], per)
            if epoch_losses is None:
                epoch_losses = {k: 0.0 for k in vals}
            for k, v in vals.items():
                epoch_losses[k] += v
        if epoch_losses is None:
            epoch_losses = {k: 0.0 for k in self.loss_tracker.train_losses}
        return {k: v / n_rows for k, v in epoch_losses.items()}

    # ------------------------------------------------------------------------------ epochs
    # ------------------------------------------------ autograd path (non-fused loss compositions)
    def _gather(self, mat, rows):
        """data = batch[0].to(float) (trainer.py:110): the batch's rows as fp32 [n, G] on the device."""
        return mat.data.index_select(0, rows.long())[:, :self.model.input_dim].float()

    def _epoch_autograd(self, loader, epoch, training):
        """trainer.py:104-156 with model(data) = libgm2's forward (VAE.forward), the components'
        compute_loss in torch, total.backward() through gm2_backward_outputs, then libgm2's clip
        statistics and Adam on the autograd gradient (L1 et al. are already in it)."""
        model = self.model
        if _dist_world() > 1:
            raise NotImplementedError("data-parallel training runs the fused loss path only (built-in components)")
        model.train(training)
        mat = loader.matrix
        batches = list(loader)
        totals = {name: 0.0 for name in (self.loss_tracker.train_losses if training else self.loss_tracker.val_losses)}
        ws = model.workspace(model.precision, loader.batch_size)
        # (a fused epoch on this workspace may have left the output-layer update deferred: it would
        # keep a pointer to model.params.grad, which zero_grad() frees -- run this loop undeferred)
        ws.join()
        ws.set_option(native.OPT_DEFER_OUTPUT_ADAM, 0)
        rec = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device=self.device)
        model.requires_grad_(training)
        try:
            for bi, rows in enumerate(batches):
                data = self._gather(mat, rows)
                eps = self._eps(rows.shape[0])
                if training:
                    model.zero_grad()
                    recon, mu, lv = model((mat, rows), eps=eps)
                    total, parts = self.loss_tracker.compute_total_loss(recon, data, mu, lv, model, epoch, bi)
                    total.backward()
                    grads = model.params.grad
                    sc = self._scalar_row({"beta": 0.0, "wgamma": 0.0, "lambda": 0.0}, self.optimizer.step_count + 1)
                    scal = torch.from_numpy(sc).to(self.device)
                    native.grad_norm(ws, model.params.detach(), grads, scal, rec)
                    native.adam_step(ws, model.params.detach(), grads, self.optimizer.exp_avg,
                                     self.optimizer.exp_avg_sq, scal)
                    self.optimizer.step_count += 1
                    model.shadows_current(model.precision)
                else:
                    with torch.no_grad():
                        recon, mu, lv = model((mat, rows), eps=eps)
                        _, parts = self.loss_tracker.compute_total_loss(recon, data, mu, lv, model, epoch, bi,
                                                                        is_training=False)
                for k, v in parts.items():
                    totals[k] += v
        finally:
            ws.join()
            model.requires_grad_(False)
            model.zero_grad()
        if training and batches:
            self.last_grad_norm = float(rec[4].item())
        n = len(loader.dataset)
        return {k: v / n for k, v in totals.items()}

    def train_epoch(self, train_loader, epoch: int) -> Dict[str, float]:
        """trainer.py:104-131. Per batch: fused fwd+bwd -> (bucketed all-reduce) -> clip stats -> Adam."""
        if not self.loss_tracker.fused:
            return self._epoch_autograd(as_strain_loader(train_loader, self.device), epoch, True)
        model = self.model
        model.train()
        loader = as_strain_loader(train_loader, self.device)
        mat = loader.matrix
        dist = get_dist()
        rank, world = rank_world(dist)
        batches = list(loader)   # draws the loader's seeds / permutation (reference order)
        for rows in batches:
            if rows.shape[0] == 1:
                raise ValueError("Expected more than 1 value per channel when training, got input size [1, "
                                 f"{model.hidden_dim}]")
        nb = len(batches)
        pers, srows = [], []
        for bi in range(nb):
            sc, per = self.loss_tracker.batch_scalars(epoch)
            pers.append(per)
            srows.append(self._scalar_row(sc, self.optimizer.step_count + bi + 1, norm_ahead=dist is None))
        scal = self._upload(srows)
        sync_bn = dist is not None and self.sync_bn
        # (rank_share gives a rank up to 3 rows of a batch smaller than 2 x world: train_rows_cap)
        ws = model.workspace(model.precision, train_rows_cap(loader.batch_size, world, sync_bn))
        rec = torch.zeros(max(nb, 1), native.LOSS_SLOTS, dtype=torch.float64, device=self.device)
        sync = self._grad_sync(dist) if dist else None
        # the output layer's Adam update runs beside the next batch's hidden layers
        # (GM2_OPT_DEFER_OUTPUT_ADAM, bit-identical; the loop below joins it before touching the
        # gradient buffer itself and at the end of the epoch). Under DDP too: the queued update reads
        # the exchanged gradient, and the next backward's output-layer bucket is written only after
        # the library has joined it (before the loss GEMM)
        ws.set_option(native.OPT_DEFER_OUTPUT_ADAM, 1)
        # (one process exchanges no gradients: no bucket events, GM2_OPT_GRAD_BUCKETS)
        ws.set_option(native.OPT_GRAD_BUCKETS, 1 if dist else 0)
        if sync:
            sync.prepare(ws)
        if sync_bn:
            enable_sync_bn(dist, ws)
        # bf16: the matrix's bf16 rows and target bits, built once and read in place by each step
        # (gm2_batch.resident: no per-batch gather)
        res = mat.operands(model.precision) if model.precision == native.GM2_BF16 else None
        for bi, rows in enumerate(batches):
            n = rows.shape[0]
            # SyncBN: plain contiguous slices (a rank may get 0 or 1 rows: the statistics are the
            # global batch's, and a rank with none still joins the 12 all-reduces inside libgm2)
            lo, hi = rank_slice(n, rank, world) if sync_bn else rank_share(n, rank, world)
            eps = self._eps(n)[lo:hi].contiguous()
            ran = hi > lo or sync_bn
            if ran:
                batch = native.make_batch(mat.data, mat.ld, rows[lo:hi], hi - lo, eps, resident=res)
                native.train_fwd_bwd(ws, batch, model.params, self.grads, model.bn, scal[bi], rec[bi])
            else:
                # DDP only: a global batch of fewer than 2 rows per rank runs on its first n // 2
                # ranks (every row is still trained, each active rank with >= 2 rows for train-mode
                # BatchNorm); this rank contributes a zero gradient and zero loss sums
                ws.join()  # (a deferred update still reads the gradient buffer)
                self.grads.zero_()
            if sync:
                sync.after_backward(ws, ran)
            native.grad_norm(ws, model.params, self.grads, scal[bi], rec[bi])
            native.adam_step(ws, model.params, self.grads, self.optimizer.exp_avg, self.optimizer.exp_avg_sq,
                             scal[bi])
            self.optimizer.step_count += 1
            model.shadows_current(model.precision)
            self._bump_bn()
        ws.join()  # (a deferred output-layer update, GM2_OPT_DEFER_OUTPUT_ADAM, if one was asked for)
        # the epoch's options end with it: later calls on this workspace (autograd forward, eval,
        # sampling on rank 0 only) neither defer an update nor issue SyncBN collectives
        ws.set_option(native.OPT_DEFER_OUTPUT_ADAM, 0)
        if sync_bn:
            ws.set_option(native.OPT_SYNC_BN, 0)
        if dist:
            reduce_loss_rows(dist, rec)
            if not sync_bn:  # (SyncBN: every rank applied the same global-batch updates)
                average_running_stats(dist, model.bn)
        raw = rec.cpu().numpy()  # the epoch's one device->host sync
        if nb:
            self.last_grad_norm = float(raw[nb - 1, 4])
        return self._epoch_values(raw, pers, len(loader.dataset))

    def validate_epoch(self, val_loader, epoch: int) -> Dict[str, float]:
        """trainer.py:133-156: eval-mode forward + the same loss components (KL counter advances)."""
        if not self.loss_tracker.fused:
            return self._epoch_autograd(as_strain_loader(val_loader, self.device), epoch, False)
        model = self.model
        model.eval()
        loader = as_strain_loader(val_loader, self.device)
        mat = loader.matrix
        dist = get_dist()
        rank, world = rank_world(dist)
        batches = list(loader)
        nb = len(batches)
        pers, srows = [], []
        for bi in range(nb):
            sc, per = self.loss_tracker.batch_scalars(epoch)
            pers.append(per)
            srows.append(self._scalar_row(sc))
        scal = self._upload(srows)
        ws = model.workspace(model.precision, (loader.batch_size + world - 1) // world)
        rec = torch.zeros(max(nb, 1), native.LOSS_SLOTS, dtype=torch.float64, device=self.device)
        for bi, rows in enumerate(batches):
            n = rows.shape[0]
            lo, hi = rank_slice(n, rank, world)
            eps = self._eps(n)[lo:hi].contiguous()
            if hi > lo:
                batch = native.make_batch(mat.data, mat.ld, rows[lo:hi], hi - lo, eps)
                native.eval_forward(ws, batch, model.params, model.bn, scal[bi], rec[bi])
        if any(isinstance(c, L1RegularizationLoss) and c.lambda_l1 for c in self.loss_tracker.loss_components) and nb:
            # parameters are constant during validation: one sum|theta| serves every batch
            native.grad_norm(ws, model.params, self.grads, scal[0], rec[0])
            rec[1:, 3] = rec[0, 3]
        if dist:
            reduce_loss_rows(dist, rec)
        raw = rec.cpu().numpy()
        return self._epoch_values(raw, pers, len(loader.dataset))

    def train(self, train_loader, val_loader, folder: str = "./") -> Tuple[List[float], List[float], int]:
        if self.loss_tracker is None:
            raise ValueError("Loss components not set up. Call setup_loss_components first.")
        epoch = 0
        for epoch in range(self.config.n_epochs):
            train_losses = self.train_epoch(train_loader, epoch)
            self.loss_tracker.update_epoch_losses(train_losses, is_training=True)
            val_losses = self.validate_epoch(val_loader, epoch)
            self.loss_tracker.update_epoch_losses(val_losses, is_training=False)
            self.scheduler.step()
            if (epoch + 1) % self.config.print_every == 0 and rank_world()[0] == 0:
                print(f"Epoch {epoch + 1}:")
                print(f"  Learning Rate: {self.scheduler.get_last_lr()[0]}")
                print(f"  Train Loss: {train_losses['total']}")
                print(f"  Validation Loss: {val_losses['total']}")
            if self.early_stopping.should_stop(val_losses["total"]):
                if rank_world()[0] == 0:
                    print(f"Early stopping triggered after {epoch + 1} epochs")
                break
        return (self.loss_tracker.train_losses["total"], self.loss_tracker.val_losses["total"], epoch + 1)


# ------------------------------------------------------------------ preset factories (trainer.py:193-257)
def create_v0_trainer(model, optimizer, scheduler, n_epochs, max_norm, beta_start, beta_end, **kw):
    t = VAETrainer(model, optimizer, scheduler, TrainingConfig(n_epochs=n_epochs, max_norm=max_norm,
                                                               lambda_l1=0.0), **kw)
    t.setup_loss_components([ReconstructionLoss(),
                             KLDivergenceLoss(scheduler_type="linear", min_beta=beta_start, max_beta=beta_end)])
    return t


def create_v1_trainer(model, optimizer, scheduler, n_epochs, max_norm, lambda_l1, beta_start=0.1, beta_end=1.0,
                      gamma_start=1.0, gamma_end=0.1, **kw):
    t = VAETrainer(model, optimizer, scheduler, TrainingConfig(n_epochs=n_epochs, max_norm=max_norm,
                                                               lambda_l1=lambda_l1), **kw)
    t.setup_loss_components([ReconstructionLoss(),
                             KLDivergenceLoss(scheduler_type="linear", min_beta=beta_start, max_beta=beta_end),
                             GeneAbundanceLoss(gamma_start=gamma_start, gamma_end=gamma_end),
                             L1RegularizationLoss(lambda_l1=lambda_l1)])
    return t


def create_v2_trainer(model, optimizer, scheduler, n_epochs, max_norm, lambda_l1, min_beta=0.0, max_beta=1.0,
                      gamma_start=1.0, gamma_end=0.1, **kw):
    t = VAETrainer(model, optimizer, scheduler, TrainingConfig(n_epochs=n_epochs, max_norm=max_norm,
                                                               lambda_l1=lambda_l1, patience=10), **kw)
    t.setup_loss_components([ReconstructionLoss(),
                             KLDivergenceLoss(scheduler_type="cosine", min_beta=min_beta, max_beta=max_beta, T=10),
                             GeneAbundanceLoss(gamma_start=gamma_start, gamma_end=gamma_end),
                             L1RegularizationLoss(lambda_l1=lambda_l1)])
    return t


def create_v3_trainer(model, optimizer, scheduler, n_epochs, max_norm, lambda_l1, min_beta=0.1, max_beta=1.0,
                      gamma_start=2.0, gamma_end=0.1, weight=1.0, **kw):
    t = VAETrainer(model, optimizer, scheduler, TrainingConfig(n_epochs=n_epochs, max_norm=max_norm,
                                                               lambda_l1=lambda_l1, patience=20, print_every=100),
                   **kw)
    t.setup_loss_components([ReconstructionLoss(),
                             KLDivergenceLoss(scheduler_type="cosine", min_beta=min_beta, max_beta=max_beta, T=50),
                             GeneAbundanceLoss(gamma_start=gamma_start, gamma_end=gamma_end, weight=weight),
                             L1RegularizationLoss(lambda_l1=lambda_l1)])
    return t


def v0(model, folder, optimizer, scheduler, n_epochs, train_loader, val_loader, beta_start, beta_end, max_norm,
       **kw):
    return create_v0_trainer(model, optimizer, scheduler, n_epochs, max_norm, beta_start, beta_end,
                             **kw).train(train_loader, val_loader, folder)


def v1(model, folder, optimizer, scheduler, n_epochs, train_loader, val_loader, beta_start, beta_end, gamma_start,
       gamma_end, max_norm, lambda_l1, **kw):
    return create_v1_trainer(model, optimizer, scheduler, n_epochs, max_norm, lambda_l1, beta_start, beta_end,
                             gamma_start, gamma_end, **kw).train(train_loader, val_loader, folder)


def v2(model, folder, optimizer, scheduler, n_epochs, train_loader, val_loader, min_beta, max_beta, gamma_start,
       gamma_end, max_norm, lambda_l1, **kw):
    return create_v2_trainer(model, optimizer, scheduler, n_epochs, max_norm, lambda_l1, min_beta, max_beta,
                             gamma_start, gamma_end, **kw).train(train_loader, val_loader, folder)


def v3(model, folder, optimizer, scheduler, n_epochs, train_loader, val_loader, min_beta, max_beta, gamma_start,
       gamma_end, weight, max_norm, lambda_l1, **kw):
    return create_v3_trainer(model, optimizer, scheduler, n_epochs, max_norm, lambda_l1, min_beta, max_beta,
                             gamma_start, gamma_end, weight, **kw).train(train_loader, val_loader, folder)


class VAETrainerBuilder:
    """trainer.py:294-372."""

    def __init__(self, model, optimizer, scheduler):
        self.model, self.optimizer, self.scheduler = model, optimizer, scheduler
        self.loss_components = []
        self.config_params = {}

    def epochs(self, n_epochs: int):
        self.config_params["n_epochs"] = n_epochs
        return self

    def gradient_clipping(self, max_norm: float):
        self.config_params["max_norm"] = max_norm
        return self

    def early_stopping(self, patience: int = 10, min_delta: float = 1e-4):
        self.config_params["patience"] = patience
        self.config_params["min_delta"] = min_delta
        return self

    def print_every(self, epochs: int):
        self.config_params["print_every"] = epochs
        return self

    def with_reconstruction_loss(self):
        self.loss_components.append(ReconstructionLoss())
        return self

    def with_kl_loss(self, scheduler_type="linear", min_beta=0.0, max_beta=1.0, T=10):
        self.loss_components.append(KLDivergenceLoss(scheduler_type=scheduler_type, min_beta=min_beta,
                                                     max_beta=max_beta, T=T))
        return self

    def with_gene_abundance_loss(self, gamma_start=0.0, gamma_end=1.0, weight=1.0):
        self.loss_components.append(GeneAbundanceLoss(gamma_start=gamma_start, gamma_end=gamma_end, weight=weight))
        return self

    def with_l1_regularization(self, lambda_l1: float):
        self.config_params["lambda_l1"] = lambda_l1
        self.loss_components.append(L1RegularizationLoss(lambda_l1=lambda_l1))
        return self

    def with_custom_loss(self, loss_component: LossComponent):
        self.loss_components.append(loss_component)
        return self

    def build(self, **kw) -> VAETrainer:
        defaults = {"n_epochs": 1, "max_norm": 1.0, "lambda_l1": 0.0, "patience": 10, "min_delta": 1e-4,
                    "print_every": 10}
        for k, v in defaults.items():
            self.config_params.setdefault(k, v)
        t = VAETrainer(self.model, self.optimizer, self.scheduler, TrainingConfig(**self.config_params), **kw)
        t.setup_loss_components(self.loss_components)
        return t


__all__ = ["VAETrainer", "VAETrainerBuilder", "TrainingConfig", "Adam", "StepLR", "create_v0_trainer",
           "create_v1_trainer", "create_v2_trainer", "create_v3_trainer", "v0", "v1", "v2", "v3"]
