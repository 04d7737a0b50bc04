"""Data-parallel VAETrainer on the GPU: world size 2 (gloo, two processes on the one MI355X, each
running libgm2) driving the real `train_epoch` / `validate_epoch` of gm2.trainer, with the
bucketed backward-overlapped gradient all-reduce of gm2.ddp.GradSync (bucket events from
gm2_wait_grad_bucket), against the oracle's per-shard math:

  * the reduced data gradient of a step == sum over the two row shards of the oracle's explicit
    gradient, each shard normalised with its OWN BatchNorm batch statistics;
    f32 path: rel 1e-4 per tensor (pre-BN Linear biases: absolute, they are rounding noise);
  * the epoch's training loss components == the oracle's per-shard sums (rel 1e-5);
  * running statistics == mean over ranks of the per-shard momentum updates, equal on both ranks;
  * parameters bit-identical on both ranks after the step (replicas stay in lock step);
  * a 3-batch validation epoch (64 + 64 + 22 rows, each split over the ranks) == the oracle's
    eval-mode losses of the same rows with the GPU's own final parameters (rel 1e-5), i.e. every
    batch row of the loss record is reduced (the round-1 strided-view bug summed the wrong ones);
  * a global batch too small to give every rank 2 rows (3 rows on 2 ranks) is trained in full on
    rank 0 (gm2.ddp.rank_share): the reduced gradient and the epoch losses are the oracle's for
    all 3 rows, as in the single-device reference (trainer.py:109-120).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from gpu_helpers import perturb_bn, synth_x
from oracle import vae_oracle as O

pytestmark = pytest.mark.gpu

G, H, L = 700, 128, 16
N_TRAIN, N_VAL, BS = 64, 150, 64
SEED = 1234
BETA_KW = dict(scheduler_type="cosine", min_beta=0.1, max_beta=1.0, T=10)
GAMMA_KW = dict(gamma_start=1.0, gamma_end=0.1, weight=1.0)
LAM = 0.01
N_EPOCHS = 10


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _state():
    torch.manual_seed(SEED)
    P = O.init_params(G, H, L)
    S = O.init_bn_state(H)
    return perturb_bn(P, S, 77)


def _data():
    return synth_x(N_TRAIN, G, 3), synth_x(N_VAL, G, 4)


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank))
    torch.set_num_threads(1)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gm2 import native
    from gm2.data import ResidentMatrix, StrainLoader
    from gm2.loss_components import GeneAbundanceLoss, KLDivergenceLoss, L1RegularizationLoss, ReconstructionLoss
    from gm2.model import VAE
    from gm2.trainer import Adam, StepLR, TrainingConfig, VAETrainer

    P, S = _state()
    m = VAE(G, H, L, precision=native.GM2_F32, init=False)
    m.load_state_dict({**P, **S})
    opt = Adam(m, lr=1e-3)
    sch = StepLR(opt, 20, 0.5)
    tr = VAETrainer(m, opt, sch, TrainingConfig(n_epochs=N_EPOCHS, max_norm=1.0, lambda_l1=LAM), eps_rng="cpu")
    tr.setup_loss_components([ReconstructionLoss(), KLDivergenceLoss(**BETA_KW), GeneAbundanceLoss(**GAMMA_KW),
                              L1RegularizationLoss(LAM)])
    xt, xv = _data()
    torch.manual_seed(SEED + 1)  # identical host RNG on both ranks: loader seeds and eps draws
    tl = StrainLoader(ResidentMatrix(xt), None, BS, shuffle=True)
    vl = StrainLoader(ResidentMatrix(xv), None, BS, shuffle=False)
    tr_losses = tr.train_epoch(tl, 0)
    torch.cuda.synchronize()
    out = dict(grads=tr.grads.cpu().numpy(), params=m.params.cpu().numpy(), bn=m.bn.cpu().numpy(),
               tr=np.array([tr_losses[k] for k in sorted(tr_losses)]))
    va_losses = tr.validate_epoch(vl, 0)
    out["va"] = np.array([va_losses[k] for k in sorted(va_losses)])
    out["keys"] = np.array(sorted(va_losses))
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), **out)
    dist.destroy_process_group()


def _shard_sums(P, S, x, eps, train):
    recon, mu, lv = O.forward(P, S, x, eps, train=train)
    bce = torch.nn.functional.binary_cross_entropy(recon, x, reduction="sum").double().item()
    return bce, recon.sum().double().item(), torch.sum(1 + lv - mu.pow(2) - lv.exp()).double().item()


def test_two_rank_trainer_epoch(tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0, r1 = np.load(tmp_path / "r0.npz"), np.load(tmp_path / "r1.npz")
    np.testing.assert_array_equal(r0["params"], r1["params"])
    np.testing.assert_array_equal(r0["bn"], r1["bn"])
    np.testing.assert_array_equal(r0["grads"], r1["grads"])
    np.testing.assert_array_equal(r0["va"], r1["va"])

    # ---- oracle: replay the trainer's host RNG use (loader base seed + sampler seed + randperm,
    # then one eps draw per batch) and the per-shard math
    P, S = _state()
    xt, xv = _data()
    torch.manual_seed(SEED + 1)
    torch.empty((), dtype=torch.int64).random_()
    perm = O.loader_perm(N_TRAIN)
    x = torch.tensor(xt[perm.numpy()], dtype=torch.float32)
    eps = torch.randn(N_TRAIN, L)
    ls = O.LossState(O.Preset("t", "cosine", 0.1, 1.0, T=10, gamma_start=1.0, gamma_end=0.1, lambda_l1=LAM),
                     N_EPOCHS)
    beta = ls.beta(0)
    gamma = ls.gamma(0)
    grads, sums, bn_new = None, np.zeros(3), {k: 0.0 for k in S if "running" in k}
    for lo, hi in ((0, N_TRAIN // 2), (N_TRAIN // 2, N_TRAIN)):
        g = O.manual_grads(P, S, x[lo:hi], eps[lo:hi], beta, gamma, 0.0)
        grads = g if grads is None else {k: grads[k] + g[k] for k in g}
        S2 = {k: v.clone() for k, v in S.items()}
        sums += np.array(_shard_sums(P, S2, x[lo:hi], eps[lo:hi], True))
        for k in bn_new:
            bn_new[k] = bn_new[k] + S2[k] / 2
    # gradient per tensor (the libgm2 layout is model.parameters() order)
    off = np.cumsum([0] + [int(np.prod(s)) for _, s in O.param_specs(G, H, L)])
    fails = []
    for i, (name, _) in enumerate(O.param_specs(G, H, L)):
        got = r0["grads"][off[i]:off[i + 1]]
        ref = grads[name].reshape(-1).numpy()
        parts = name.split(".")
        if parts[0] in ("encoder", "decoder") and parts[1] in ("0", "3", "6") and parts[2] == "bias":
            scale = float(np.abs(grads[name.replace("bias", "weight")].numpy()).max())
            if np.abs(got).max() > 1e-3 * scale:
                fails.append(f"{name}: |g| {np.abs(got).max():.3g} vs weight scale {scale:.3g}")
            continue
        e = float(np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-30))
        if e > 1e-4:
            fails.append(f"{name}: rel err {e:.3g}")
    assert not fails, "\n".join(fails)
    # running statistics: mean of the two shards' momentum updates
    for i, b in enumerate(O.BNS):
        np.testing.assert_allclose(r0["bn"][i, 0], bn_new[b + ".running_mean"].numpy(), rtol=2e-5, atol=2e-6)
        np.testing.assert_allclose(r0["bn"][i, 1], bn_new[b + ".running_var"].numpy(), rtol=2e-5, atol=2e-6)
    # training losses of the epoch (one batch): components from the summed shard values
    keys = list(r0["keys"])
    tr = dict(zip(keys, r0["tr"]))
    l1 = sum(v.abs().sum().item() for v in P.values())
    exp = {"reconstruction": sums[0] / N_TRAIN, "gene_abundance": np.float32(gamma) * sums[1] / N_TRAIN,
           "kl_divergence": np.float32(beta) * (-0.5 * sums[2]) / N_TRAIN,
           "l1_regularization": LAM * l1 / N_TRAIN}
    for k, v in exp.items():
        assert abs(tr[k] - v) <= 1e-5 * abs(v) + 1e-7, (k, tr[k], v)

    # ---- validation epoch with the GPU's own final parameters and averaged running statistics
    Pf = O.unflatten(r0["params"], G, H, L)
    Sf = {k: v.clone() for k, v in S.items()}
    for i, b in enumerate(O.BNS):
        Sf[b + ".running_mean"] = torch.tensor(r0["bn"][i, 0])
        Sf[b + ".running_var"] = torch.tensor(r0["bn"][i, 1])
    torch.empty((), dtype=torch.int64).random_()  # the val loader's base seed
    xv_t = torch.tensor(xv, dtype=torch.float32)
    vs = np.zeros(3)
    betas, n_b = [], 0
    for s0 in range(0, N_VAL, BS):
        xb = xv_t[s0:s0 + BS]
        eb = torch.randn(xb.shape[0], L)
        betas.append(ls.beta(0))
        bce, ps, kl = _shard_sums(Pf, Sf, xb, eb, False)
        vs += [bce, np.float32(gamma) * ps, np.float32(betas[-1]) * (-0.5 * kl)]
        n_b += 1
    va = dict(zip(keys, r0["va"]))
    assert n_b == 3
    for k, v in zip(["reconstruction", "gene_abundance", "kl_divergence"], vs):
        assert abs(va[k] - v / N_VAL) <= 1e-5 * abs(v / N_VAL) + 1e-7, (k, va[k], v / N_VAL)


def _exchange_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank))
    torch.set_num_threads(1)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gm2 import native
    from gm2.data import ResidentMatrix
    from gm2.ddp import GradSync
    from gm2.model import VAE

    Gx, Hx, Lx, Bx = 20000, 1024, 32, 128
    x = synth_x(Bx, Gx, 20 + rank)  # each rank its own rows
    torch.manual_seed(SEED)
    m = VAE(Gx, Hx, Lx, precision=native.GM2_BF16)
    ws = m.workspace(native.GM2_BF16, Bx)
    mat = ResidentMatrix(x)
    eps = torch.randn(Bx, Lx, generator=torch.Generator().manual_seed(rank)).cuda()
    sc = torch.zeros(native.NUM_SCALARS, dtype=torch.float32, device="cuda")
    sc[native.S_BETA] = 0.5
    res = {}
    for ex in ("f32", "bf16"):
        grads = torch.zeros_like(m.params)
        loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device="cuda")
        sync = GradSync(dist, m, grads, exchange=ex)
        sync.prepare(ws)
        native.train_fwd_bwd(ws, native.make_batch(mat.data, mat.ld, None, Bx, eps), m.params, grads, m.bn, sc, loss)
        sync.after_backward(ws)
        torch.cuda.synchronize()
        res[ex] = grads.cpu().numpy()
    np.savez(os.path.join(out_dir, f"x{rank}.npz"), **res, bounds=np.array(sync.bounds))
    dist.destroy_process_group()


def test_two_rank_bf16_gradient_exchange(tmp_path):
    """GradSync(exchange="bf16"): the decoder.9 / encoder.0 weight buckets travel and are summed in
    bf16, the rest in fp32. Both ranks end with the same gradient; the bf16 buckets are within bf16
    rounding of the fp32 exchange (a few 2^-9 of the tensor's max |g|), the fp32 bucket identical."""
    port = _free_port()
    mp.spawn(_exchange_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0, r1 = np.load(tmp_path / "x0.npz"), np.load(tmp_path / "x1.npz")
    np.testing.assert_array_equal(r0["bf16"], r1["bf16"])
    np.testing.assert_array_equal(r0["f32"], r1["f32"])
    b = r0["bounds"]
    for k, (lo, hi) in enumerate(b):
        ref, got = r0["f32"][lo:hi], r0["bf16"][lo:hi]
        if k == 1:
            np.testing.assert_array_equal(got, ref)
        else:
            assert np.abs(got - ref).max() <= 4 * 2.0 ** -9 * np.abs(ref).max()


def _ragged_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank))
    torch.set_num_threads(1)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gm2 import native
    from gm2.data import ResidentMatrix, StrainLoader
    from gm2.loss_components import KLDivergenceLoss, ReconstructionLoss
    from gm2.model import VAE
    from gm2.trainer import Adam, StepLR, TrainingConfig, VAETrainer

    P, S = _state()
    m = VAE(G, H, L, precision=native.GM2_F32, init=False)
    m.load_state_dict({**P, **S})
    opt = Adam(m, lr=1e-3)
    tr = VAETrainer(m, opt, StepLR(opt, 20, 0.5), TrainingConfig(n_epochs=N_EPOCHS, max_norm=1.0), eps_rng="cpu")
    tr.setup_loss_components([ReconstructionLoss(), KLDivergenceLoss(scheduler_type="linear", min_beta=0.1,
                                                                     max_beta=1.0)])
    x3 = synth_x(3, G, 5)
    torch.manual_seed(SEED + 2)
    losses = tr.train_epoch(StrainLoader(ResidentMatrix(x3), None, BS, shuffle=False), 0)
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"g{rank}.npz"), grads=tr.grads.cpu().numpy(), params=m.params.cpu().numpy(),
             rec=np.array([losses["reconstruction"], losses["kl_divergence"]]))
    dist.destroy_process_group()


def test_two_rank_ragged_batch_trains_every_row(tmp_path):
    port = _free_port()
    mp.spawn(_ragged_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0, r1 = np.load(tmp_path / "g0.npz"), np.load(tmp_path / "g1.npz")
    np.testing.assert_array_equal(r0["params"], r1["params"])
    np.testing.assert_array_equal(r0["grads"], r1["grads"])
    P, S = _state()
    x = torch.tensor(synth_x(3, G, 5), dtype=torch.float32)
    torch.manual_seed(SEED + 2)
    torch.empty((), dtype=torch.int64).random_()  # the loader's base seed
    eps = torch.randn(3, L)
    beta = O.LossState(O.Preset("t", "linear", 0.1, 1.0), N_EPOCHS).beta(0)
    # exact (fp64) gradient of all 3 rows, and the reference's own fp32 arithmetic (torch CPU)
    g64 = O.manual_grads({k: v.double() for k, v in P.items()}, {k: v.double() for k, v in S.items()}, x.double(),
                         eps.double(), beta, 0.0, 0.0)
    g32 = O.manual_grads(P, S, x, eps, beta, 0.0, 0.0)
    off = np.cumsum([0] + [int(np.prod(s)) for _, s in O.param_specs(G, H, L)])
    # the trainer's grads buffer holds the reduced data gradient of the step (before clip / Adam);
    # bar: the C2 method (norm-wise error vs exact <= 3x the reference arithmetic's + 2e-4)
    for i, (name, _) in enumerate(O.param_specs(G, H, L)):
        parts = name.split(".")
        if parts[0] in ("encoder", "decoder") and parts[1] in ("0", "3", "6") and parts[2] == "bias":
            continue
        ex = g64[name].reshape(-1).numpy()
        nrm = max(float(np.linalg.norm(ex)), 1e-30)
        f_gpu = float(np.linalg.norm(r0["grads"][off[i]:off[i + 1]] - ex)) / nrm
        f_ref = float(np.linalg.norm(g32[name].reshape(-1).double().numpy() - ex)) / nrm
        assert f_gpu <= 3 * f_ref + 2e-4, (name, f_gpu, f_ref)
    bce, _, kl = _shard_sums(P, {k: v.clone() for k, v in S.items()}, x, eps, True)
    assert abs(r0["rec"][0] - bce / 3) <= 1e-5 * abs(bce / 3)
    assert abs(r0["rec"][1] - np.float32(beta) * (-0.5 * kl) / 3) <= 1e-5 * abs(kl) + 1e-7


def _syncbn_worker(rank, world, port, out_dir, n_rows):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank))
    torch.set_num_threads(1)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gm2 import native
    from gm2.data import ResidentMatrix, StrainLoader
    from gm2.loss_components import GeneAbundanceLoss, KLDivergenceLoss, ReconstructionLoss
    from gm2.model import VAE
    from gm2.trainer import Adam, StepLR, TrainingConfig, VAETrainer

    P, S = _state()
    m = VAE(G, H, L, precision=native.GM2_F32, init=False)
    m.load_state_dict({**P, **S})
    opt = Adam(m, lr=1e-3)
    tr = VAETrainer(m, opt, StepLR(opt, 20, 0.5), TrainingConfig(n_epochs=N_EPOCHS, max_norm=1.0), eps_rng="cpu",
                    sync_bn=True)
    tr.setup_loss_components([ReconstructionLoss(), KLDivergenceLoss(**BETA_KW), GeneAbundanceLoss(**GAMMA_KW)])
    x = synth_x(n_rows, G, 8)
    torch.manual_seed(SEED + 3)
    losses = tr.train_epoch(StrainLoader(ResidentMatrix(x), None, BS, shuffle=False), 0)
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"s{rank}.npz"), grads=tr.grads.cpu().numpy(), params=m.params.cpu().numpy(),
             bn=m.bn.cpu().numpy(), rec=np.array([losses["reconstruction"], losses["kl_divergence"],
                                                 losses["gene_abundance"]]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_rows", [(2, 64), (2, 3), (3, 2)])
def test_sync_bn_step_equals_full_batch_reference(tmp_path, world, n_rows):
    """SyncBN (gm2.ddp.enable_sync_bn, GM2_OPT_SYNC_BN): one global batch of n_rows split over
    `world` ranks (64 rows on 2; 3 rows = 1 + 2; 2 rows on 3 ranks, one rank with NO rows that only
    joins the all-reduces) gives the single-device reference's step on the WHOLE batch: the reduced
    gradient against the fp64 full-batch oracle with the C2 method's bar (norm-wise error <= 3x
    the reference's own fp32 arithmetic + 2e-4), the BatchNorm running statistics equal to the
    full-batch update on every rank (no averaging), the epoch losses equal to the full-batch sums,
    all ranks identical."""
    port = _free_port()
    mp.spawn(_syncbn_worker, args=(world, port, str(tmp_path), n_rows), nprocs=world, join=True)
    rs = [np.load(tmp_path / f"s{r}.npz") for r in range(world)]
    for r in rs[1:]:
        np.testing.assert_array_equal(rs[0]["params"], r["params"])
        np.testing.assert_array_equal(rs[0]["grads"], r["grads"])
        np.testing.assert_array_equal(rs[0]["bn"], r["bn"])
    P, S = _state()
    x = torch.tensor(synth_x(n_rows, G, 8), dtype=torch.float32)
    torch.manual_seed(SEED + 3)
    torch.empty((), dtype=torch.int64).random_()  # the loader's base seed
    eps = torch.randn(n_rows, L)
    ls = O.LossState(O.Preset("t", "cosine", 0.1, 1.0, T=10, gamma_start=1.0, gamma_end=0.1), N_EPOCHS)
    beta, gamma = ls.beta(0), ls.gamma(0)
    P64 = {k: v.double() for k, v in P.items()}
    S64 = {k: v.double() for k, v in S.items()}
    g64 = O.manual_grads(P64, S64, x.double(), eps.double(), beta, gamma, 0.0)
    g32 = O.manual_grads(P, S, x, eps, beta, gamma, 0.0)
    off = np.cumsum([0] + [int(np.prod(s)) for _, s in O.param_specs(G, H, L)])
    fails = []
    for i, (name, _) in enumerate(O.param_specs(G, H, L)):
        parts = name.split(".")
        if parts[0] in ("encoder", "decoder") and parts[1] in ("0", "3", "6") and parts[2] == "bias":
            continue
        ex = g64[name].reshape(-1).numpy()
        nrm = max(float(np.linalg.norm(ex)), 1e-30)
        f_gpu = float(np.linalg.norm(rs[0]["grads"][off[i]:off[i + 1]] - ex)) / nrm
        f_ref = float(np.linalg.norm(g32[name].reshape(-1).double().numpy() - ex)) / nrm
        if not f_gpu <= 3 * f_ref + 2e-4:
            fails.append(f"{name}: fro {f_gpu:.3g} vs reference arithmetic {f_ref:.3g}")
    assert not fails, "\n".join(fails)
    S2 = {k: v.clone() for k, v in S64.items()}
    O.forward(P64, S2, x.double(), eps.double(), train=True)
    for i, b in enumerate(O.BNS):
        np.testing.assert_allclose(rs[0]["bn"][i, 0], S2[b + ".running_mean"].numpy(), rtol=2e-5, atol=2e-6)
        np.testing.assert_allclose(rs[0]["bn"][i, 1], S2[b + ".running_var"].numpy(), rtol=2e-5, atol=2e-6)
    bce, ps, kl = _shard_sums(P64, {k: v.clone() for k, v in S64.items()}, x.double(), eps.double(), True)
    np.testing.assert_allclose(rs[0]["rec"][0], bce / n_rows, rtol=1e-5)
    np.testing.assert_allclose(rs[0]["rec"][1], np.float32(beta) * (-0.5 * kl) / n_rows, rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(rs[0]["rec"][2], np.float32(gamma) * ps / n_rows, rtol=1e-5)


def _sample_worker(rank, world, port, root, ckpt, pkl, n):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK="0", GM2_DIST_BACKEND="gloo")
    torch.set_num_threads(1)
    import main as cli
    torch.manual_seed(4321)  # rank 0's draw of the shared seed
    rc = cli.main(["--mode", "sample", "--model-path", ckpt, "--genes-path", pkl, "--num-samples", str(n),
                   "--project-root", root, "--no-csv"])
    assert rc == 0


def test_two_rank_sharded_sampling_cli(tmp_path):
    """`--mode sample` under torchrun (2 ranks, gloo, one GPU): one broadcast seed, the same z on
    both ranks, each rank decodes its contiguous half, rank 0 gathers the packed masks and writes
    the reference's .npy. The file holds exactly the masks of decoding that z on one device:
    bit-exact to the fp32 oracle outside the fp64 rounding band of each logit."""
    import pickle
    from gm2.data import write_synthetic_csvs
    root = str(tmp_path)
    Gs, Hs, Ls, n = 300, 1024, 64, 1001
    write_synthetic_csvs(root, 50, Gs, seed=6)
    torch.manual_seed(11)
    Pq = O.init_params(Gs, Hs, Ls)
    Sq = O.init_bn_state(Hs)
    Pq, Sq = perturb_bn(Pq, Sq, 12)
    Pq["decoder.9.bias"] = torch.linspace(-1.5, 1.0, Gs)
    sd = {**Pq, **Sq}
    for b in O.BNS:
        sd[b + ".num_batches_tracked"] = torch.tensor(0, dtype=torch.long)
    ckpt = os.path.join(root, "saved_VAE_v0.pt")
    torch.save(sd, ckpt)
    pkl = os.path.join(root, "ess.pkl")
    with open(pkl, "wb") as f:
        pickle.dump({"a": [0, 3], "b": [299]}, f)
    port = _free_port()
    mp.spawn(_sample_worker, args=(2, port, root, ckpt, pkl, n), nprocs=2, join=True)
    masks = np.load(os.path.join(root, "models", "v0_model", "sampling_results", "v0_binary_samples_default.npy"))
    assert masks.shape == (n, Gs)
    torch.manual_seed(4321)
    seed = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())
    torch.cuda.manual_seed(seed)
    z = torch.randn(n, Ls, device="cuda").cpu()
    ref = O.sample_decode(Pq, Sq, z).numpy() > 0.5
    band = np.abs(O.decode_logits64(Pq, Sq, z).numpy()) <= 1e-3
    assert ((masks.astype(bool) != ref) & ~band).sum() == 0


def _small_batch_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank))
    torch.set_num_threads(1)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gm2 import native
    from gm2.data import ResidentMatrix, StrainLoader
    from gm2.loss_components import KLDivergenceLoss, ReconstructionLoss
    from gm2.model import VAE
    from gm2.trainer import Adam, StepLR, TrainingConfig, VAETrainer

    P, S = _state()
    m = VAE(G, H, L, precision=native.GM2_F32, init=False)
    m.load_state_dict({**P, **S})
    opt = Adam(m, lr=1e-3)
    tr = VAETrainer(m, opt, StepLR(opt, 20, 0.5), TrainingConfig(n_epochs=N_EPOCHS, max_norm=1.0), eps_rng="cpu")
    tr.setup_loss_components([ReconstructionLoss(), KLDivergenceLoss(scheduler_type="linear", min_beta=0.1,
                                                                     max_beta=1.0)])
    torch.manual_seed(SEED + 3)
    # batch_size 4 on 3 ranks, 7 rows: batches of 4 (2 + 2 rows on ranks 0-1) and 3 (all on rank 0)
    losses = tr.train_epoch(StrainLoader(ResidentMatrix(synth_x(7, G, 9)), None, 4, shuffle=True), 0)
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"s{rank}.npz"), params=m.params.cpu().numpy(),
             rec=np.array([losses["reconstruction"], losses["kl_divergence"]]))
    dist.destroy_process_group()


def test_three_rank_batch_smaller_than_two_per_rank(tmp_path):
    """a global batch of at most 2 x world rows, with a ragged last batch (4, then 3 rows
    on 3 ranks): rank_share gives one rank all 3 rows of the last batch, more than ceil(4 / 3); the
    trainer sizes its workspace with gm2.ddp.train_rows_cap, so the epoch runs, and every rank ends
    with the same parameters and loss record."""
    port = _free_port()
    mp.spawn(_small_batch_worker, args=(3, port, str(tmp_path)), nprocs=3, join=True)
    r = [np.load(tmp_path / f"s{k}.npz") for k in range(3)]
    for k in (1, 2):
        np.testing.assert_array_equal(r[0]["params"], r[k]["params"])
        np.testing.assert_array_equal(r[0]["rec"], r[k]["rec"])
    assert np.isfinite(r[0]["rec"]).all() and np.isfinite(r[0]["params"]).all()


def _xchg_worker(rank, world, port, out_dir, n):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    import torch.distributed as dist
    from gm2.ddp import bf16_exchange_sum
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(500 + rank)
    x = torch.randn(n, generator=g) * torch.exp(2.0 * torch.randn(n, generator=g)) * 1e-3
    x[::53] = 0.0
    dev = bf16_exchange_sum(dist, x.cuda(), {})    # libgm2's pack / rank-order sum / unpack kernels
    host = bf16_exchange_sum(dist, x.clone(), {})  # the same method in torch (the CPU form)
    np.save(os.path.join(out_dir, f"d{rank}.npy"), dev.cpu().numpy())
    np.save(os.path.join(out_dir, f"h{rank}.npy"), host.numpy())
    dist.destroy_process_group()


def test_two_rank_bf16_exchange_kernels_bit_equal_to_torch(tmp_path):
    """gm2.ddp.bf16_exchange_sum on device tensors runs the cast, the rank-order fp32 sum and the
    widening as libgm2 kernels (gm2_exchange_pack / _ranksum / _unpack); over 2 ranks (gloo, both on
    the one GPU) the result equals the torch form of the same method bit for bit, on both ranks."""
    n = (1 << 17) + 37
    port = _free_port()
    mp.spawn(_xchg_worker, args=(2, port, str(tmp_path), n), nprocs=2, join=True)
    for r in range(2):
        np.testing.assert_array_equal(np.load(tmp_path / f"d{r}.npy"), np.load(tmp_path / f"h{r}.npy"))
    np.testing.assert_array_equal(np.load(tmp_path / "d0.npy"), np.load(tmp_path / "d1.npy"))


def test_exchange_kernels_against_torch_single_process():
    """The three exchange entry points directly, world 3 and a ragged length: pack == torch's RNE cast
    with zero pad, ranksum == ((p0 + p1) + p2) in fp32 then RNE, unpack == the exact widening."""
    from gm2 import native
    n, world = 100_003, 3
    c = -(-n // world)
    c = -(-c // 8) * 8
    x = (torch.randn(world * c) * torch.exp(3.0 * torch.randn(world * c))).cuda()
    x[::17] = 0.0
    send = torch.empty(world * c, dtype=torch.bfloat16, device="cuda")
    native.exchange_pack(x[:n], send)
    ref = torch.zeros(world * c, dtype=torch.bfloat16, device="cuda")
    ref[:n] = x[:n].to(torch.bfloat16)
    assert torch.equal(send.view(torch.int16), ref.view(torch.int16))
    parts = x.to(torch.bfloat16)
    out = torch.empty(c, dtype=torch.bfloat16, device="cuda")
    native.exchange_ranksum(parts, world, out)
    acc = parts[:c].float()
    for r in range(1, world):
        acc = acc + parts[r * c:(r + 1) * c].float()
    assert torch.equal(out.view(torch.int16), acc.to(torch.bfloat16).view(torch.int16))
    y = torch.empty(n - 5, device="cuda")
    native.exchange_unpack(parts, y)
    assert torch.equal(y, parts[:n - 5].float())
