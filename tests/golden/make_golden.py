#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by IMPORTING the reference.

Run here (the build container) only — `/root/reference` does not exist on the GPU box:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What it imports (read-only, never modified, no bytecode written):
  * src/genome_minimizer_2/training/model.py                 (VAE, model.py:13-120)
  * src/genome_minimizer_2/training/training/trainer.py      (VAETrainer, v0..v3, trainer.py:84-290)
  * src/genome_minimizer_2/training/training/loss_components (loss_components.py:46-202)
`utils/extras.py` and `utils/experiments.py` are NOT importable here (they import seaborn, and
`data_exploration.py:39-41` mkdirs under the reference's PROJECT_ROOT at import time), so the three
lines of `sample_from_model` (extras.py:192-203) and the two `train_test_split` calls of
`create_dataloaders` (experiments.py:232-237) are driven from here against the reference's own
`VAE.decode` / sklearn, exactly as those call sites do.

Every fixture records torch.__version__ and the thread count (1): reference training is
bit-deterministic only at a fixed thread count. It also records the CPU model, the
ATen dispatch level and MKL_CBWR=COMPATIBLE, the MKL code path the fixtures were made on: MKL's
default path differs between Intel and AMD hosts (1-ulp differences in every GEMM), COMPATIBLE is
the same on both, and tests/conftest.py selects it for the CPU suite.

Outputs are small .npz files (inputs + expected outputs, i.e. data, no reference source).
"""
import json
import math
import os
import sys

import numpy as np

REF = "/root/reference"
OUT = os.environ.get("GM2_GOLDEN_OUT") or os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
# MKL picks its sgemm code path per CPU vendor/ISA, so the reference's fp32 bits differ between an
# Intel and an AMD host by ~1 ulp. The COMPATIBLE branch (conditional numerical reproducibility) is
# the one MKL honours on every x86 vendor; it must be set before the first MKL call.
os.environ["MKL_CBWR"] = "COMPATIBLE"

import torch  # noqa: E402

torch.set_num_threads(1)

from src.genome_minimizer_2.training.model import VAE  # noqa: E402
from src.genome_minimizer_2.training.training import trainer as T  # noqa: E402
from src.genome_minimizer_2.training.training import loss_components as LC  # noqa: E402
from torch.utils.data import DataLoader, TensorDataset  # noqa: E402
from sklearn.model_selection import train_test_split  # noqa: E402

def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


META = {"torch": torch.__version__, "threads": 1, "numpy": np.__version__,
        "generator": "tests/golden/make_golden.py", "cpu": _cpu_model(),
        "aten_cpu_capability": torch.backends.cpu.get_cpu_capability(),
        "mkl_cbwr": os.environ["MKL_CBWR"]}

PRESET_HP = {
    # experiments.py:42-114 (hyper-parameters only; dims are shrunk for fixtures)
    "v0": dict(min_beta=0.1, max_beta=1.0, lambda_l1=0.0),
    "v1": dict(min_beta=0.1, max_beta=1.0, gamma_start=1.0, gamma_end=0.1, lambda_l1=0.01),
    "v2": dict(min_beta=0.0, max_beta=1.0, gamma_start=1.0, gamma_end=0.1, lambda_l1=0.01),
    "v3": dict(min_beta=0.1, max_beta=1.0, gamma_start=2.0, gamma_end=0.1, weight=1.0,
               lambda_l1=0.01),
}


def synth_matrix(n, g, seed):
    """Pan-genome-like binary matrix: 15% core genes at f=0.98, accessory f~Beta(0.1,1)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    f = rng.beta(0.1, 1.0, size=g)
    core = rng.random(g) < 0.15
    f[core] = 0.98
    return (rng.random((n, g)) < f[None, :]).astype(np.uint8)


def flat_params(model):
    return np.concatenate([p.detach().reshape(-1).numpy() for p in model.parameters()])


def flat_grads(model):
    return np.concatenate([p.grad.detach().reshape(-1).numpy() for p in model.parameters()])


def bn_state(model):
    sd = model.state_dict()
    keys = [k for k in sd if k.endswith("running_mean") or k.endswith("running_var")]
    return np.concatenate([sd[k].reshape(-1).numpy() for k in keys]), keys


def state_npz(model, prefix):
    return {prefix + k: v.detach().numpy().copy() for k, v in model.state_dict().items()}


def make_trainer(preset, model, opt, sched, n_epochs):
    hp = PRESET_HP[preset]
    if preset == "v0":
        return T.create_v0_trainer(model, opt, sched, n_epochs, 1.0, hp["min_beta"], hp["max_beta"])
    if preset == "v1":
        return T.create_v1_trainer(model, opt, sched, n_epochs, 1.0, hp["lambda_l1"], hp["min_beta"],
                                   hp["max_beta"], hp["gamma_start"], hp["gamma_end"])
    if preset == "v2":
        return T.create_v2_trainer(model, opt, sched, n_epochs, 1.0, hp["lambda_l1"], hp["min_beta"],
                                   hp["max_beta"], hp["gamma_start"], hp["gamma_end"])
    return T.create_v3_trainer(model, opt, sched, n_epochs, 1.0, hp["lambda_l1"], hp["min_beta"],
                               hp["max_beta"], hp["gamma_start"], hp["gamma_end"], hp["weight"])


def gen_init():
    """Reference init at several dims (model.py:62-120): pins the host-side init RNG replay."""
    out = {}
    for tag, (g, h, l, seed) in {"a": (37, 64, 16, 0), "b": (200, 64, 16, 7)}.items():
        torch.manual_seed(seed)
        m = VAE(g, h, l)
        out[f"{tag}_dims"] = np.array([g, h, l, seed])
        out[f"{tag}_params"] = flat_params(m)
        # RNG state after construction: the next draw must match too
        out[f"{tag}_next"] = torch.rand(4).numpy()
    np.savez_compressed(os.path.join(OUT, "init.npz"), meta=json.dumps(META), **out)


def gen_steps():
    """One-batch training steps per preset (trainer.py:104-131 through the reference)."""
    G, H, L, B, EPOCH, NEP = 150, 64, 16, 48, 3, 10
    out = {"dims": np.array([G, H, L, B, EPOCH, NEP])}
    X = synth_matrix(B, G, 11)
    out["X"] = X
    for pi, preset in enumerate(["v0", "v1", "v2", "v3"]):
        torch.manual_seed(100 + pi)
        model = VAE(G, H, L)
        if pi == 0:
            out["init_params"] = flat_params(model)
        init_sd = {k: v.clone() for k, v in model.state_dict().items()}
        opt = torch.optim.Adam(model.parameters(), lr=1e-3)
        sched = torch.optim.lr_scheduler.StepLR(opt, step_size=20, gamma=0.5)
        tr = make_trainer(preset, model, opt, sched, NEP)
        # advance cosine counters as if 5 earlier calls happened (exercise t = epoch*32+counter)
        for c in tr.loss_tracker.loss_components:
            if isinstance(c, LC.KLDivergenceLoss):
                c.counter = 5
        loader = DataLoader(TensorDataset(torch.tensor(X, dtype=torch.float32)), batch_size=B,
                            shuffle=False)
        rng_before = torch.get_rng_state()
        losses = tr.train_epoch(loader, EPOCH)
        # epsilon drawn by randn_like inside reparameterization (model.py:102). The DataLoader
        # iterator draws one int64 base seed from the global generator first.
        after = torch.get_rng_state()
        torch.set_rng_state(rng_before)
        torch.empty((), dtype=torch.int64).random_()
        rng_eps = torch.get_rng_state()
        eps = torch.randn(B, L)
        torch.set_rng_state(after)
        out[f"{preset}_init_seed"] = np.array([100 + pi])
        out[f"{preset}_eps"] = eps.numpy()
        names = [c.get_name() for c in tr.loss_tracker.loss_components] + ["total"]
        out[f"{preset}_loss_names"] = np.array(names)
        out[f"{preset}_losses"] = np.array([losses[n] * B for n in names], dtype=np.float64)
        out[f"{preset}_grads"] = flat_grads(model)  # clipped (+L1) grads after the step
        out[f"{preset}_params"] = flat_params(model)
        st = opt.state
        out[f"{preset}_exp_avg"] = np.concatenate(
            [st[p]["exp_avg"].reshape(-1).numpy() for p in model.parameters()])
        out[f"{preset}_exp_avg_sq"] = np.concatenate(
            [st[p]["exp_avg_sq"].reshape(-1).numpy() for p in model.parameters()])
        bn, keys = bn_state(model)
        out[f"{preset}_bn"] = bn
        if pi == 0:
            out["bn_keys"] = np.array(keys)
        # unclipped data gradient at the INITIAL params, for kernel-level checks
        m2 = VAE(G, H, L)
        m2.load_state_dict(init_sd)
        m2.train()
        torch.set_rng_state(rng_eps)
        xt = torch.tensor(X, dtype=torch.float32)
        recon, mu, lv = m2(xt)
        tr2 = make_trainer(preset, m2, torch.optim.Adam(m2.parameters()), None, NEP)
        for c in tr2.loss_tracker.loss_components:
            if isinstance(c, LC.KLDivergenceLoss):
                c.counter = 5
        tot, ind = tr2.loss_tracker.compute_total_loss(recon, xt, mu, lv, m2, EPOCH, 0)
        tot.backward()
        for n in names:
            assert ind[n] == losses[n] * B or abs(ind[n] - losses[n] * B) <= 1e-9 * abs(ind[n]), n
        out[f"{preset}_raw_grads"] = flat_grads(m2)
        out[f"{preset}_mu"] = mu.detach().numpy()
        out[f"{preset}_logvar"] = lv.detach().numpy()
        torch.set_rng_state(after)
    np.savez_compressed(os.path.join(OUT, "steps.npz"), meta=json.dumps(META), **out)


def gen_trainer():
    """Whole preset functions v0..v3 (trainer.py:261-290) for 3 epochs with a shuffled loader,
    StepLR and validation: pins epoch loop, shuffle RNG use, val eps draws, cosine counter."""
    G, H, L, N, BS, NEP = 120, 64, 16, 150, 32, 3
    data = synth_matrix(N, G, 21).astype(np.float32)
    idx = np.arange(N)
    tr_idx, tmp_idx = train_test_split(idx, test_size=0.3, random_state=12345)
    va_idx, te_idx = train_test_split(tmp_idx, test_size=0.3333, random_state=12345)
    out = {"dims": np.array([G, H, L, N, BS, NEP]), "data": data.astype(np.uint8),
           "train_idx": tr_idx, "val_idx": va_idx, "test_idx": te_idx}
    for pi, preset in enumerate(["v0", "v1", "v2", "v3"]):
        torch.manual_seed(200 + pi)
        model = VAE(G, H, L)
        opt = torch.optim.Adam(model.parameters(), lr=1e-3)
        sched = torch.optim.lr_scheduler.StepLR(opt, step_size=20, gamma=0.5)
        tl = DataLoader(TensorDataset(torch.tensor(data[tr_idx])), batch_size=BS, shuffle=True)
        vl = DataLoader(TensorDataset(torch.tensor(data[va_idx])), batch_size=BS, shuffle=False)
        hp = PRESET_HP[preset]
        if preset == "v0":
            res = T.v0(model, "./", opt, sched, NEP, tl, vl, hp["min_beta"], hp["max_beta"], 1.0)
        elif preset == "v1":
            res = T.v1(model, "./", opt, sched, NEP, tl, vl, hp["min_beta"], hp["max_beta"],
                       hp["gamma_start"], hp["gamma_end"], 1.0, hp["lambda_l1"])
        elif preset == "v2":
            res = T.v2(model, "./", opt, sched, NEP, tl, vl, hp["min_beta"], hp["max_beta"],
                       hp["gamma_start"], hp["gamma_end"], 1.0, hp["lambda_l1"])
        else:
            res = T.v3(model, "./", opt, sched, NEP, tl, vl, hp["min_beta"], hp["max_beta"],
                       hp["gamma_start"], hp["gamma_end"], hp["weight"], 1.0, hp["lambda_l1"])
        out[f"{preset}_seed"] = np.array([200 + pi])
        out[f"{preset}_train_losses"] = np.array(res[0], dtype=np.float64)
        out[f"{preset}_val_losses"] = np.array(res[1], dtype=np.float64)
        out[f"{preset}_epochs"] = np.array([res[2]])
        out[f"{preset}_params"] = flat_params(model)
        out[f"{preset}_bn"] = bn_state(model)[0]
        out[f"{preset}_nbt"] = np.array([int(v) for k, v in model.state_dict().items()
                                         if k.endswith("num_batches_tracked")])
        out[f"{preset}_rng_after"] = torch.rand(3).numpy()
    np.savez_compressed(os.path.join(OUT, "trainer.npz"), meta=json.dumps(META), **out)


def gen_sampling():
    """sample_from_model (extras.py:192-203) + focused mode (main.py:351-370) driven against the
    reference VAE.decode on CPU, eval mode, after load_state_dict (extras.py:185-187)."""
    out = {}
    for tag, (G, H, L, N, seed) in {"s": (200, 64, 16, 256, 3), "p": (300, 256, 32, 64, 4)}.items():
        torch.manual_seed(seed)
        model = VAE(G, H, L)
        # give BN non-trivial running stats + a shifted decoder so masks are not ~50/50 noise
        with torch.no_grad():
            for i, mod in enumerate(model.modules()):
                if isinstance(mod, torch.nn.BatchNorm1d):
                    mod.running_mean.uniform_(-0.2, 0.2)
                    mod.running_var.uniform_(0.5, 1.5)
                    mod.weight.uniform_(0.8, 1.2)
                    mod.bias.uniform_(-0.1, 0.1)
            model.decoder[9].bias.uniform_(-2.0, 1.0)
        model.eval()
        torch.manual_seed(1000 + seed)
        with torch.no_grad():
            z = torch.randn(N, L)
            p = model.decode(z).numpy()
        binary = (p > 0.5).astype(float)
        out[f"{tag}_dims"] = np.array([G, H, L, N])
        # decode-only fixture: the encoder/heads are not on the decode path; keep decoder.* only
        out.update({k: v for k, v in state_npz(model, f"{tag}_sd/").items() if "/decoder." in k})
        out[f"{tag}_z"] = z.numpy()
        out[f"{tag}_p"] = p
        out[f"{tag}_mask"] = binary.astype(np.uint8)
        # fp64 logits: certify the masks (|logit| margin) for the bit-exact GPU test
        with torch.no_grad():
            md = VAE(G, H, L).double()
            md.load_state_dict({k: (v.double() if v.is_floating_point() else v)
                                for k, v in model.state_dict().items()})
            md.eval()
            h = md.decoder[:9](z.double())
            logit64 = md.decoder[9](h).numpy()
        out[f"{tag}_logit64"] = logit64
        # focused sampling, main.py:351-370, noise 0.1, N samples
        torch.manual_seed(2000 + seed)
        with torch.no_grad():
            zt = torch.randn(100, L)
            ct = model.decode(zt).numpy()
        bt = (ct > 0.5).astype(float)
        mi = np.argmin(bt.sum(axis=1))
        ci = np.argmin(np.linalg.norm(ct - ct[mi], axis=1))
        with torch.no_grad():
            noise = torch.randn(N, L) * 0.1
            zf = zt[ci].unsqueeze(0) + noise
            cf = model.decode(zf).numpy()
        out[f"{tag}_focused_idx"] = np.array([mi, ci])
        out[f"{tag}_focused_mask"] = (cf > 0.5).astype(np.uint8)
        out[f"{tag}_focused_z"] = zf.numpy()
    np.savez_compressed(os.path.join(OUT, "sampling.npz"), meta=json.dumps(META), **out)


def gen_numerics():
    """Element-level semantics: sigmoid threshold (extras.py:200-201), BCE clamps + backward
    (loss_components.py:49-50), KL/abundance schedules (loss_components.py:76-115, 187-202)."""
    out = {}
    # threshold: fp32 bit patterns around 0 and around 0x33C00000
    bits = np.concatenate([np.arange(0x33B00000, 0x33D00000, 97, dtype=np.uint32),
                           np.arange(0, 0x00100000, 4099, dtype=np.uint32),
                           np.arange(0x80000000, 0x80100000, 4099, dtype=np.uint32),
                           np.array([0x33BFFFFF, 0x33C00000, 0x33C00001], dtype=np.uint32)])
    xs = bits.view(np.float32)
    out["thr_x"] = xs
    out["thr_mask"] = (torch.sigmoid(torch.tensor(xs)).numpy() > 0.5).astype(np.uint8)
    # BCE through the reference's ReconstructionLoss on sigmoid(logit), autograd grads
    logits = np.concatenate([np.linspace(-40, 40, 161, dtype=np.float32),
                             np.array([-103.0, -90.0, -88.7, 16.5, 17.0, 30.0, 89.0], np.float32)])
    for tgt in (0, 1):
        l = torch.tensor(logits, requires_grad=True)
        p = torch.sigmoid(l)
        x = torch.full_like(p, float(tgt))
        loss = LC.ReconstructionLoss().compute_loss(p, x, None, None, None, 0, 0)
        loss.backward()
        out[f"bce_loss_t{tgt}"] = np.array([loss.item()], dtype=np.float32)
        out[f"bce_grad_t{tgt}"] = l.grad.numpy().copy()
        elem = []
        for v in logits:
            lv = torch.tensor([v])
            pv = torch.sigmoid(lv)
            elem.append(LC.ReconstructionLoss().compute_loss(pv, torch.full_like(pv, float(tgt)),
                                                             None, None, None, 0, 0).item())
        out[f"bce_elem_t{tgt}"] = np.array(elem, dtype=np.float32)
    out["bce_logits"] = logits
    # schedules: kl_loss == 1 exactly with mu = sqrt(2), logvar = 0 -> returns beta
    mu = torch.tensor([[math.sqrt(2.0)]], dtype=torch.float64)
    lv = torch.zeros_like(mu)
    rows = []
    for (st, lo, hi, Tp, nep) in [("linear", 0.1, 1.0, 10, 7), ("cosine", 0.0, 1.0, 10, 7),
                                  ("cosine", 0.1, 1.0, 50, 7), ("constant", 0.1, 0.7, 10, 7)]:
        kl = LC.KLDivergenceLoss(scheduler_type=st, min_beta=lo, max_beta=hi, T=Tp)
        kl.n_epochs = nep
        for epoch in range(4):
            for _ in range(3):
                b = kl.compute_loss(None, None, mu, lv, None, epoch, 0).item()
                rows.append(b)
    out["sched_beta"] = np.array(rows, dtype=np.float64)
    ga = LC.GeneAbundanceLoss(gamma_start=2.0, gamma_end=0.1, weight=1.5)
    ga.n_epochs = 9
    one = torch.ones(1, 1, dtype=torch.float64)
    out["sched_gamma"] = np.array([ga.compute_loss(one, None, None, None, None, e, 0).item()
                                   for e in range(12)], dtype=np.float64)
    # split sizes (experiments.py:232-237) for several N
    sizes = []
    for n in (10, 150, 1000, 7512, 10000):
        a, b = train_test_split(np.arange(n), test_size=0.3, random_state=12345)
        c, d = train_test_split(b, test_size=0.3333, random_state=12345)
        sizes.append([n, len(a), len(c), len(d), int(a[:5].sum()), int(c[:5].sum()), int(d[:5].sum())])
        if n == 1000:
            out["split1000_train"], out["split1000_val"], out["split1000_test"] = a, c, d
    out["split_sizes"] = np.array(sizes)
    np.savez_compressed(os.path.join(OUT, "numerics.npz"), meta=json.dumps(META), **out)


if __name__ == "__main__":
    gen_init()
    gen_steps()
    gen_trainer()
    gen_sampling()
    gen_numerics()
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))
