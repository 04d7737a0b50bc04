"""CPU-only checks: the C-ABI library loads and exports what include/gm2.h declares, its host-side
queries (layouts, sizes, argument validation) work without a GPU, and the host mirror of the
reference interface (init RNG replay, loader RNG, schedules, loss bookkeeping) matches the goldens."""
import os
import re

import numpy as np
import pytest
import torch

from golden_io import load

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    txt = open(os.path.join(ROOT, "include", "gm2.h")).read()
    return sorted(set(re.findall(r"\b(gm2_[a-z_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from gm2 import native
    lib = native.lib()
    names = _declared()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
    assert sorted(native.EXPORTS) == names


def test_header_constants_match_binding():
    """The ctypes mirror (gm2/native.py) uses the values include/gm2.h defines: ABI version, gradient
    bucket count, option keys, the gm2_batch field order (ABI 2 adds `next`); option setters accept
    and reject values without a GPU, and the bucket bounds tile the gradient buffer in order. ABI 3:
    options and bucket events are per workspace; a workspace libgm2 never initialised is refused.
    ABI 4: gm2_batch gains the resident-operand fields; gm2_resident_layout sizes them. ABI 5: seven
    tuning options pruned (their keys now refused), the sampling decode's GM2_STAT_* counters. ABI 6:
    band-list overflow recomputed whole per block (GM2_STAT_OVERFLOW_TILES), the list capacity and the
    single tier's gate as workspace options."""
    import ctypes
    from gm2 import native
    txt = open(os.path.join(ROOT, "include", "gm2.h")).read()
    assert int(re.search(r"#define GM2_ABI_VERSION (\d+)", txt).group(1)) == native.lib().gm2_abi_version() \
        == native.ABI_VERSION == 6
    bogus = ctypes.c_void_p(0x1000)
    v = ctypes.c_int()
    assert native.lib().gm2_workspace_set_option(bogus, native.OPT_GRID_CAP, 1) != 0
    assert "not initialised" in native.lib().gm2_last_error().decode()
    assert native.lib().gm2_workspace_get_option(bogus, native.OPT_GRID_CAP, ctypes.byref(v)) != 0
    assert native.lib().gm2_wait_grad_bucket(bogus, 0, None) != 0
    assert native.lib().gm2_workspace_release(bogus) == 0  # releasing unknown state is a no-op
    assert int(re.search(r"#define GM2_GRAD_BUCKETS (\d+)", txt).group(1)) == native.GRAD_BUCKETS
    opts = dict((k, int(v)) for k, v in re.findall(r"GM2_OPT_([A-Z_]+) = (\d+)", txt))
    for k, v in opts.items():
        assert getattr(native, "OPT_" + k) == v, k
    stats = dict((k, int(v)) for k, v in re.findall(r"GM2_STAT_([A-Z_]+) = (\d+)", txt))
    assert len(stats) == 9 and set(native.DECODE_STATS.values()) == set(stats.values())
    for k, v in stats.items():
        assert getattr(native, "STAT_" + k) == v, k
    assert [f[0] for f in native.Batch._fields_] == ["data", "ld_data", "rows", "n", "eps", "next", "resident",
                                                     "ld_resident", "resident_bits", "ld_resident_bits",
                                                     "resident_rows", "resident_prec"]
    # (the header's struct fields, in order)
    body = re.search(r"typedef struct gm2_batch \{(.*?)\} gm2_batch;", txt, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = re.findall(r"(\w+);", body)
    assert fields == [f[0] for f in native.Batch._fields_]
    ld, ldb, rows = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    nb, nbb = ctypes.c_size_t(), ctypes.c_size_t()
    assert native.lib().gm2_resident_layout(10000, 55039, native.GM2_BF16, ctypes.byref(ld), ctypes.byref(ldb),
                                            ctypes.byref(rows), ctypes.byref(nb), ctypes.byref(nbb)) == 0
    assert (ld.value, ldb.value, rows.value) == (55040, 1720, 10048)
    assert nb.value == 10048 * 55040 * 2 and nbb.value == 10048 * 1720 * 4
    assert native.lib().gm2_resident_layout(-1, 5, native.GM2_BF16, ctypes.byref(ld), ctypes.byref(ldb),
                                            ctypes.byref(rows), ctypes.byref(nb), ctypes.byref(nbb)) != 0
    native.set_option(native.OPT_INPUT_CHUNKS, 4)
    assert native.get_option(native.OPT_INPUT_CHUNKS) == 4
    native.set_option(native.OPT_INPUT_CHUNKS, 1)
    with pytest.raises(RuntimeError, match="1 or 4"):
        native.set_option(native.OPT_INPUT_CHUNKS, 2)
    with pytest.raises(RuntimeError, match="4 or 8"):
        native.set_option(native.OPT_SMALL_WAVES, 5)
    native.set_option(native.OPT_SAMPLE_BAND_CAP, 7)
    assert native.get_option(native.OPT_SAMPLE_BAND_CAP) == 7
    native.set_option(native.OPT_SAMPLE_BAND_CAP, 65536)
    with pytest.raises(RuntimeError, match="band list cap"):
        native.set_option(native.OPT_SAMPLE_BAND_CAP, 65537)
    with pytest.raises(RuntimeError, match="single-tier bound"):
        native.set_option(native.OPT_SAMPLE_SINGLE_BOUND, 0)
    assert native.get_option(native.OPT_SAMPLE_SINGLE_BOUND) == 250
    # the options pruned in ABI 5 (measured slower or neutral; evidence kept in profiles/) are gone
    for key in (8, 12, 13, 14, 16, 17, 19, 23):  # (23: round 6's GM2_OPT_SMALL_PAIR, measured and removed)
        with pytest.raises(RuntimeError, match="unknown option"):
            native.set_option(key, 0)
    G, H, L = 55039, 1024, 64
    b = native.grad_bucket_bounds(native.dims(G, H, L, 4096))
    cover = sorted(b)
    assert cover[0][0] == 0 and cover[-1][1] == native.param_offsets(G, H, L)[-1]
    assert all(cover[i][1] == cover[i + 1][0] for i in range(len(cover) - 1))


def test_process_default_options_from_env():
    """GM2_OPTS="key=value,..." (options.hip) sets process defaults at library load for same-box A/Bs:
    valid entries apply, a refused value and an unknown key are ignored, parsing stops at garbage."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, 'genome-minimizer-2_amd'); from gm2 import native as n; "
            "print(n.get_option(n.OPT_SMALL_WAVES), n.get_option(n.OPT_SMALL_SPLIT), n.get_option(n.OPT_GRID_CAP), "
            "n.get_option(n.OPT_SAMPLE_SINGLE))")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GM2_OPTS="6=4,4=3,9=99,999=1,20=0,x,6=8")
    out = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    # 6=4 and 4=3 applied, 9=99 refused (grid cap stays 3), 999 unknown, 20=0 applied, "x" ends parsing
    assert out.stdout.split() == ["4", "3", "3", "0"], out.stdout


def test_layout_queries_and_errors():
    from gm2 import native
    G, H, L = 55039, 1024, 64
    off = native.param_offsets(G, H, L)
    assert off[-1] == 117184383  # P(v0, G=55,039), SURVEY.md §8a-a1
    assert native.param_offsets(20000, 1024, 64)[-1] == 45389472
    assert native.param_offsets(55039, 512, 32)[-1] == 57521983
    ws = native.workspace_size(native.dims(G, H, L, 4096), native.GM2_BF16)
    assert 1e9 < ws < 16e9
    with pytest.raises(RuntimeError, match="multiple of 128"):
        native.workspace_size(native.dims(100, 100, 16, 32), native.GM2_F32)
    with pytest.raises(RuntimeError, match="divide 256"):
        native.workspace_size(native.dims(100, 128, 48, 32), native.GM2_F32)


def test_param_specs_match_reference_order():
    from gm2.model import param_specs
    from oracle import vae_oracle as O
    assert param_specs(37, 64, 16) == O.param_specs(37, 64, 16)
    from gm2 import native
    off = native.param_offsets(150, 128, 16)
    sizes = [int(np.prod(s)) for _, s in param_specs(150, 128, 16)]
    assert list(np.diff(off)) == sizes


def test_reference_init_replay():
    from gm2.model import reference_init
    g = load("init")
    for tag in ("a", "b"):
        G, H, L, seed = [int(v) for v in g[f"{tag}_dims"]]
        torch.manual_seed(seed)
        flat = torch.cat([t.reshape(-1) for t in reference_init(G, H, L)]).numpy()
        np.testing.assert_array_equal(flat, g[f"{tag}_params"])
        np.testing.assert_array_equal(torch.rand(4).numpy(), g[f"{tag}_next"])


def test_loader_rng_matches_torch_dataloader():
    """StrainLoader consumes the global generator exactly as DataLoader(shuffle=True/False)."""
    from torch.utils.data import DataLoader, TensorDataset

    from gm2.data import StrainLoader

    class FakeMatrix:
        n = 101
        data = torch.zeros(1)

    X = torch.arange(101, dtype=torch.float32)[:, None]
    for shuffle in (True, False):
        torch.manual_seed(5)
        ref = [b[0][:, 0].long().tolist() for b in DataLoader(TensorDataset(X), batch_size=16, shuffle=shuffle)]
        after_ref = torch.rand(2)
        torch.manual_seed(5)
        sl = StrainLoader(FakeMatrix(), None, 16, shuffle)
        got = [b.long().tolist() for b in sl]
        np.testing.assert_array_equal(torch.rand(2).numpy(), after_ref.numpy())
        assert got == ref


def test_schedules_and_loss_values():
    from gm2 import loss_components as LC
    g = load("numerics")
    rows = []
    for (st, lo, hi, Tp, nep) in [("linear", 0.1, 1.0, 10, 7), ("cosine", 0.0, 1.0, 10, 7),
                                  ("cosine", 0.1, 1.0, 50, 7), ("constant", 0.1, 0.7, 10, 7)]:
        kl = LC.KLDivergenceLoss(scheduler_type=st, min_beta=lo, max_beta=hi, T=Tp)
        kl.n_epochs = nep
        for epoch in range(4):
            for _ in range(3):
                rows.append(kl.scalars(epoch)["beta"])
    np.testing.assert_allclose(rows, g["sched_beta"], rtol=1e-15, atol=0)
    ga = LC.GeneAbundanceLoss(gamma_start=2.0, gamma_end=0.1, weight=1.5)
    ga.n_epochs = 9
    np.testing.assert_allclose([ga.scalars(e)["wgamma"] for e in range(12)], g["sched_gamma"], rtol=1e-15)


@pytest.mark.parametrize("preset", ["v0", "v1", "v2", "v3"])
def test_batch_loss_bookkeeping(preset):
    """Per-batch fp32 component values rebuilt from raw device sums reproduce the reference's
    .item() values bit-for-bit (trainer.py:44-56) when the raw sums equal the reference's."""
    from gm2 import loss_components as LC
    from gm2.trainer import LossTracker
    from oracle import vae_oracle as O
    g = load("steps")
    G, H, L, B, EPOCH, NEP = [int(v) for v in g["dims"]]
    torch.manual_seed(int(g[f"{preset}_init_seed"][0]))
    P = O.init_params(G, H, L)
    S = O.init_bn_state(H)
    x = torch.tensor(g["X"], dtype=torch.float32)
    eps = torch.tensor(g[f"{preset}_eps"])
    recon, mu, lv = O.forward(P, S, x, eps, train=True)
    raw = np.zeros(8)
    raw[0] = torch.nn.functional.binary_cross_entropy(recon, x, reduction="sum").item()
    raw[1] = torch.sum(torch.abs(recon.sum(axis=0))).item()
    raw[2] = torch.sum(1 + lv - mu.pow(2) - lv.exp()).item()
    raw[3] = sum(torch.sum(torch.abs(v)).item() for v in P.values()) if False else 0.0
    pen = 0.0
    for v in P.values():
        pen += torch.sum(torch.abs(v))
    raw[3] = pen.item()
    pr = O.PRESETS[preset]
    comps = [LC.ReconstructionLoss(),
             LC.KLDivergenceLoss(pr.kl_type, pr.min_beta, pr.max_beta, pr.T)]
    if pr.gamma_start is not None:
        comps.append(LC.GeneAbundanceLoss(pr.gamma_start, pr.gamma_end, pr.weight))
    if pr.lambda_l1 is not None:
        comps.append(LC.L1RegularizationLoss(pr.lambda_l1))
    for c in comps:
        if hasattr(c, "n_epochs"):
            c.n_epochs = NEP
        if isinstance(c, LC.KLDivergenceLoss):
            c.counter = 5
    lt = LossTracker(comps)
    sc, per = lt.batch_scalars(EPOCH)
    vals = lt.batch_values(raw, per)
    names = list(g[f"{preset}_loss_names"])
    got = np.array([vals[n] for n in names], dtype=np.float32)
    np.testing.assert_array_equal(got, g[f"{preset}_losses"].astype(np.float32))


def test_early_stopping_semantics():
    from gm2.trainer import EarlyStopping
    es = EarlyStopping(patience=2, min_delta=1e-4)
    assert not es.should_stop(1.0)
    assert not es.should_stop(0.99995)   # not better by min_delta
    assert es.should_stop(0.99999)
    es = EarlyStopping(patience=2, min_delta=1e-4)
    seq = [5.0, 4.0, 4.0, 3.0, 3.0, 3.0]
    assert [es.should_stop(v) for v in seq] == [False, False, False, False, False, True]


def test_steplr():
    from gm2.trainer import StepLR

    class O:
        param_groups = [{"lr": 1e-3}]
    s = StepLR(O(), step_size=20, gamma=0.5)
    lrs = []
    for _ in range(45):
        lrs.append(s.get_last_lr()[0])
        s.step()
    assert lrs[0] == 1e-3 and lrs[19] == 1e-3 and lrs[20] == 5e-4 and lrs[40] == 2.5e-4


def test_count_essential_genes_matches_reference_loop():
    """Vectorised count_essential_genes == the reference's loop (oracle restatement of
    extras.py:49-87) on 0/1, uint8, bool and fractional masks, with single, multiple, empty,
    out-of-range and negative positions."""
    from gm2.extras import count_essential_genes
    from oracle import vae_oracle as O
    rng = np.random.Generator(np.random.PCG64(4))
    G = 40
    pos = {"a": [3], "b": [5, 39], "c": [], "d": [41], "e": [41, 7], "f": [-1], "g": [0, 1, 2]}
    x = (rng.random((25, G)) < 0.3)
    for m in (x.astype(np.float64), x.astype(np.uint8), x, rng.random((25, G)) * 1.5):
        np.testing.assert_array_equal(count_essential_genes(m, pos), O.count_essential_genes_loop(m, pos))
