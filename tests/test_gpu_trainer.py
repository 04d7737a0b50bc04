"""Trainer- and CLI-level parity on the GPU: whole v0..v3 runs (shuffled loader, eval pass, KL
counter, StepLR, early-stopping bookkeeping) through libgm2 in exact fp32 against the CPU oracle's
restatement of trainer.py:158-189 (oracle/vae_oracle.py:run_preset, itself pinned bit-exact to
tests/golden/trainer.npz), and `main.py --mode training|sample` end to end on synthetic CSVs."""
import os
import pickle

import numpy as np
import pytest
import torch

from gm2 import native
from gpu_helpers import rel_err
from oracle import vae_oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _prebn_bias_names():
    # Linear biases feeding a train-mode BatchNorm: their gradient is rounding noise in the
    # reference too (BN removes any per-column shift), so Adam moves them by noise-driven steps.
    return {"encoder.0.bias", "encoder.3.bias", "encoder.6.bias", "decoder.0.bias", "decoder.3.bias",
            "decoder.6.bias"}


def _no_constant_columns(n, g, seed):
    """Synthetic rows whose gene frequencies stay <= 0.7. A gene present in EVERY row of a batch
    gives encoder.0.weight a gradient column that is exactly zero in real arithmetic (BatchNorm's
    backward makes each column of dY sum to zero) and pure rounding noise in fp32; without an L1 term
    (v0) Adam normalises that noise into +-lr steps, so two correct fp32 implementations (or the
    reference at two thread counts) drift apart by O(lr) per step on those weights. Parity over whole
    runs is therefore checked on data without such columns (0.7^32 ~ 1e-5 per column and batch)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    f = np.minimum(rng.beta(0.5, 1.0, size=g), 0.7)
    return (rng.random((n, g)) < f[None, :]).astype(np.uint8)


def _oracle_run(preset, dtype, seed, x, tr_idx, va_idx, G, H, L, NEP, BS):
    torch.manual_seed(seed)
    P = {k: v.to(dtype) for k, v in O.init_params(G, H, L).items()}
    S = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in O.init_bn_state(H).items()}
    xt = torch.tensor(x, dtype=dtype)
    tr, va, ep = O.run_preset(P, S, O.PRESETS[preset], NEP, xt[tr_idx], xt[va_idx], BS)
    return np.array(tr), np.array(va), ep, P, S, torch.rand(3)


@pytest.mark.parametrize("preset", ["v0", "v1", "v2", "v3"])
def test_preset_run_matches_oracle(preset):
    """Whole-run parity. Over several Adam steps fp32 rounding is amplified chaotically on a few
    weights (Adam divides small, cancellation-dominated gradients by their own RMS), so the oracle's
    fp32 run is itself off its fp64 run by up to ~2e-3 on some elements (v1 here). The bar is
    therefore relative to exact arithmetic: the GPU run (exact fp32 MFMA) must be at least about as
    close to the fp64 oracle as the fp32 oracle is (x2), on losses and on every parameter except
    the six pre-BN Linear biases, whose gradients are pure rounding noise in any implementation."""
    from gm2.data import ResidentMatrix, StrainLoader
    from gm2.experiments import PRESETS, run_preset
    from gm2.model import VAE
    from gm2.trainer import Adam, StepLR
    G, H, L, N, BS, NEP = 200, 128, 16, 150, 32, 3
    x = _no_constant_columns(N, G, 11)
    tr_idx, va_idx = np.arange(0, 96), np.arange(96, 126)   # whole batches only (no short batch)
    # seed 301 (v1) hits such a ReLU-boundary event at step 5 (kept as the example in the comment
    # below); the run-level comparison uses seeds where the fp32 and fp64 oracles agree to 1e-4
    seed = {"v0": 300, "v1": 311, "v2": 302, "v3": 303}[preset]
    o32 = _oracle_run(preset, torch.float32, seed, x, tr_idx, va_idx, G, H, L, NEP, BS)
    o64 = _oracle_run(preset, torch.float64, seed, x, tr_idx, va_idx, G, H, L, NEP, BS)
    # libgm2 (GPU, exact fp32 GEMMs), eps drawn on the CPU generator as the CPU reference does
    torch.manual_seed(seed)
    m = VAE(G, H, L, precision=native.GM2_F32)
    mat = ResidentMatrix(x)
    cfg = PRESETS[preset]()
    cfg.n_epochs, cfg.hidden_dim, cfg.latent_dim = NEP, H, L
    opt = Adam(m, lr=cfg.learning_rate)
    sch = StepLR(opt, step_size=cfg.scheduler_step_size, gamma=cfg.scheduler_gamma)
    tr, va, ep = run_preset(cfg, m, opt, sch, StrainLoader(mat, tr_idx, BS, True),
                            StrainLoader(mat, va_idx, BS, False), eps_rng="cpu")
    after = torch.rand(3)
    assert ep == o32[2] == o64[2]
    np.testing.assert_array_equal(after.numpy(), o32[5].numpy())  # same RNG consumption
    # The six pre-BN Linear biases (6H values) random-walk on rounding noise: their data gradient
    # is zero in exact arithmetic, so Adam's normalisation (and, for v1-v3, the sign of the L1
    # gradient at 0) decides their path differently in every fp32 implementation, fp64 keeping
    # them near 0. They do not change any training-mode output, but they enter (a) the L1 loss
    # value lambda*sum|theta| of every batch and (b) validation through BatchNorm running means.
    # (a) is bounded explicitly: per batch at most lambda * 6H * 2*lr*steps.
    lam = O.PRESETS[preset].lambda_l1 or 0.0
    nb = -(-len(tr_idx) // BS)
    steps = nb * np.arange(1, NEP + 1)
    allow_tr = lam * nb * 6 * H * 2 * 1e-3 * steps / len(tr_idx)
    d_gpu, d_ref = np.abs(np.array(tr) - o64[0]), np.abs(o32[0] - o64[0])
    print(f"{preset} train loss |diff| vs fp64 oracle: gpu {d_gpu}, fp32 oracle {d_ref}, L1 allowance {allow_tr}")
    assert (d_gpu <= 2 * d_ref + allow_tr + 2e-7 * np.abs(o64[0])).all()
    # (b): validation losses within 1e-4 relative (measured ~1e-5, the fp32 oracle's own ~2e-5)
    e_gpu, e_ref = rel_err(va, o64[1]), rel_err(o32[1], o64[1])
    print(f"{preset} val loss rel vs fp64 oracle: gpu {e_gpu:.2e}, fp32 oracle {e_ref:.2e}")
    assert e_gpu <= max(2 * e_ref, 1e-4)
    # Parameters. A ReLU pre-activation that lands within rounding of 0 in some row flips that
    # unit's gradient for the row (seen here: v1 step 5, fp32 vs fp64 oracle, encoder unit 17),
    # after which a few percent of the weights take a different O(lr) Adam path in whichever
    # implementations fell on the other side -- the fp32 oracle on some CPUs included. So: the bulk
    # (>= 97 % of elements) within 2x the fp32 oracle's own distance to fp64 (floor 2e-5), and
    # every element within Adam's bound of 2*lr per step.
    sd = m.state_dict()
    skip = _prebn_bias_names()
    names = [k for k in o64[3] if k not in skip]
    d_gpu = torch.cat([(sd[k].cpu().double() - o64[3][k]).abs().reshape(-1) for k in names])
    d_ref = torch.cat([(o32[3][k].double() - o64[3][k]).abs().reshape(-1) for k in names])
    tight = max(2 * float(d_ref.max()), 2e-5)
    frac = float((d_gpu > tight).double().mean())
    print(f"{preset} |param - fp64 oracle|: gpu max {float(d_gpu.max()):.2e}, fp32 oracle max "
          f"{float(d_ref.max()):.2e}; fraction beyond {tight:.1e}: gpu {frac:.4f}, "
          f"fp32 oracle {float((d_ref > tight).double().mean()):.4f}")
    assert frac <= 0.03
    assert float(d_gpu.max()) <= 2 * 1e-3 * nb * NEP
    for i, b in enumerate(O.BNS):
        assert m.num_batches_tracked[i] == int(o32[4][b + ".num_batches_tracked"])
        assert rel_err(sd[b + ".running_var"].cpu(), o64[4][b + ".running_var"]) <= 1e-4


def test_cli_training_then_sampling(tmp_path, capsys):
    import main as cli
    from gm2.data import write_synthetic_csvs
    root = str(tmp_path)
    x = write_synthetic_csvs(root, 96, 300, seed=5)
    rc = cli.main(["--mode", "training", "--preset", "v0", "--epochs", "2", "--project-root", root,
                   "--precision", "f32"])
    assert rc == 0
    ckpt = os.path.join(root, "models", "trained_models", "v0_model", "saved_VAE_v0.pt")
    sd = torch.load(ckpt, weights_only=True, map_location="cpu")
    assert sd["encoder.0.weight"].shape == (1024, 300) and sd["decoder.9.bias"].shape == (300,)
    assert int(sd["encoder.1.num_batches_tracked"]) == 2 * 3  # 67 train rows / batch 32 -> 3 batches
    # sampling from that checkpoint: masks equal the fp32 oracle's outside the rounding band
    pos = {"geneA": [0, 5], "geneB": [7], "geneC": [299, 1000]}
    pkl = os.path.join(root, "ess.pkl")
    with open(pkl, "wb") as f:
        pickle.dump(pos, f)
    torch.manual_seed(1234)
    rc = cli.main(["--mode", "sample", "--model-path", ckpt, "--genes-path", pkl, "--num-samples", "40",
                   "--project-root", root])
    assert rc == 0
    out = os.path.join(root, "models", "v0_model", "sampling_results")
    masks = np.load(os.path.join(out, "v0_binary_samples_default.npy"))
    assert masks.dtype == np.float64 and masks.shape == (40, 300)
    torch.manual_seed(1234)
    z = torch.randn(40, 64, device="cuda").cpu()
    P = {k: v for k, v in sd.items() if not k.endswith(("running_mean", "running_var", "num_batches_tracked"))}
    S = {k: v for k, v in sd.items() if k.endswith(("running_mean", "running_var", "num_batches_tracked"))}
    ref = (O.sample_decode(P, S, z).numpy() > 0.5)
    band = np.abs(O.decode_logits64(P, S, z).numpy()) <= 1e-3
    assert ((masks.astype(bool) != ref) & ~band).sum() == 0
    import pandas as pd
    df = pd.read_csv(os.path.join(out, "v0_data_full_samples_df.csv"))
    assert df.shape == (300, 41) and df.columns[0] == "Gene"
    assert x.shape == (96, 300)
    # --mask-dtype bits: the same masks packed (numpy packbits, bitorder little); the printed
    # statistics come from the device (sizes, essential counts) and convert-samples reads the file
    capsys.readouterr()
    torch.manual_seed(1234)
    rc = cli.main(["--mode", "sample", "--model-path", ckpt, "--genes-path", pkl, "--num-samples", "40",
                   "--project-root", root, "--mask-dtype", "bits", "--no-csv"])
    assert rc == 0
    printed = capsys.readouterr().out
    bits = np.load(os.path.join(out, "v0_binary_samples_default.npy"))
    assert bits.dtype == np.uint8 and bits.shape == (40, (300 + 7) // 8)
    np.testing.assert_array_equal(np.unpackbits(bits, axis=1, count=300, bitorder="little"), masks.astype(np.uint8))
    from gm2.extras import count_essential_genes
    ess = count_essential_genes(masks, pos)
    assert f"- Median essential genes: {np.median(ess):.0f}" in printed
    assert f"- Median genome size: {np.median(masks.sum(axis=1)):.0f} genes" in printed
    ids_out = os.path.join(root, "ids.npy")
    assert cli.main(["--mode", "convert-samples", "--genes-path", os.path.join(out, "v0_binary_samples_default.npy"),
                     "--output-file", ids_out, "--project-root", root]) == 0
    ids = np.load(ids_out, allow_pickle=True)  # written by our own code just above
    genes = [f"gene{i:05d}" for i in range(300)]
    assert [list(r) for r in ids] == [[genes[j] for j in np.flatnonzero(r)] for r in masks]
