"""Device consumers of the sampled masks on packed masks in HBM:

  * decode_bits: the packed masks of gm2_decode_bits == numpy packbits(bitorder='little') of the u8
    masks of gm2_decode_mask (same decode, bit-exact) at a ragged G and a ragged N;
  * count_essential_genes on the device == the REFERENCE's counts (tests/golden/essential.npz,
    produced by the reference's own function), incl. multi-position genes, positions >= G,
    negative positions, astype(int) truncation;
  * gene-index CSR (masks_to_gene_lists' compaction) == numpy nonzero, with and without a keep mask;
    the converter goldens (tests/golden/converter.json, produced by importing the reference's
    binary_converter.py) through the device path;
  * calculate_reconstruction_metrics == sklearn's f1_score / accuracy_score on the oracle's fp32
    reconstruction with the same noise (band-free fixture: no logit within 1e-4 of the threshold).
All integer / index results bit-exact.
"""
import json
import os

import numpy as np
import pandas as pd
import pytest
import torch

from golden_io import load
from gpu_helpers import oracle_state, perturb_bn, synth_x, to_model
from oracle import vae_oracle as O

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from gm2 import native
    from gm2.masks import PackedMasks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("G,N", [(1000, 300), (3001, 1029)])
def test_decode_bits_matches_decode_mask(G, N):
    H, L = 128, 16
    P, S = perturb_bn(*oracle_state(G, H, L, 70), seed=71)
    P["decoder.9.bias"] = torch.linspace(-1.0, 1.0, G)
    m = to_model(P, S, G, H, L, native.GM2_F32)
    m.eval()
    z = torch.randn(N, L)
    mask, _ = m.decode_mask(z)
    pm, _ = m.decode_bits(z, chunk=512)
    u8 = mask.cpu().numpy()
    np.testing.assert_array_equal(pm.to_host(), np.packbits(u8, axis=1, bitorder="little"))
    np.testing.assert_array_equal(pm.unpack(), u8)
    np.testing.assert_array_equal(pm.row_sizes(), u8.sum(axis=1))
    assert pm.bits[:, (G + 7) // 8:].sum().item() == 0  # pad bytes stay zero


@pytest.mark.parametrize("name", ["u8", "f64", "frac", "bool"])
def test_count_essential_on_device_matches_reference(name):
    from gm2.extras import count_essential_genes
    g = load("essential")
    masks = g[f"{name}_masks"]
    offs, pos = g[f"{name}_offsets"], g[f"{name}_positions"]
    d = {f"g{i}": [int(p) for p in pos[offs[i]:offs[i + 1]]] for i in range(len(offs) - 1)}
    pm = PackedMasks.from_host(masks.astype(int) != 0, threshold=True)  # the reference's astype(int) test
    np.testing.assert_array_equal(count_essential_genes(pm, d), g[f"{name}_counts"])


@pytest.mark.parametrize("G,N,ngroups", [(55039, 1000, 300), (1000, 130, 900), (4100, 70, 0)])
def test_count_groups_whole_row_kernel(G, N, ngroups):
    """gm2_mask_count_groups (whole-row form: single-position groups through an LDS bit mask, the
    rest listed) == a numpy count of the reference's rule (a group counts when any of its positions
    is set) with single-position groups on distinct and on shared genes, multi-position groups,
    empty groups and positions at the row's last bits; G = 1000 with 900 groups puts most groups on
    genes another group already holds."""
    rng = np.random.Generator(np.random.PCG64(G + ngroups))
    M = rng.random((N, G)) < 0.3
    M[0] = True
    M[1] = False
    groups = []
    for i in range(ngroups):
        k = int(rng.integers(0, 4)) if i % 7 else 1
        groups.append([int(x) for x in rng.integers(0, G, size=k)])
    if ngroups:
        groups[0] = [G - 1]
        groups[1] = [G - 1]  # the same gene again
        groups[2] = []
    offs = np.concatenate([[0], np.cumsum([len(x) for x in groups])]).astype(np.int32)
    pos = np.array([p for x in groups for p in x] or [0], dtype=np.int32)
    want = np.zeros(N, dtype=np.int32)
    for x in groups:
        if x:
            want += M[:, x].any(axis=1)
    pm = PackedMasks.from_host(M, threshold=True)
    counts = torch.zeros(N, dtype=torch.int32, device="cuda")
    native.mask_count_groups(pm.bits, N, pm.bits.shape[1], torch.from_numpy(offs).cuda(), ngroups,
                             torch.from_numpy(pos).cuda(), counts)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(counts.cpu().numpy(), want)


def test_gene_index_csr_vs_numpy():
    rng = np.random.Generator(np.random.PCG64(5))
    M = rng.random((777, 4100)) < 0.3
    M[5] = False
    M[6] = True
    pm = PackedMasks.from_host(M, threshold=True)
    offs, idx = pm.gene_index_csr()
    nz = np.nonzero(M)
    np.testing.assert_array_equal(offs, np.concatenate([[0], np.cumsum(M.sum(axis=1))]))
    np.testing.assert_array_equal(idx, nz[1])
    keep = rng.random(4100) < 0.9
    offs, idx = pm.gene_index_csr(keep)
    Mk = M & keep[None, :]
    np.testing.assert_array_equal(offs, np.concatenate([[0], np.cumsum(Mk.sum(axis=1))]))
    np.testing.assert_array_equal(idx, np.nonzero(Mk)[1])


def test_converter_goldens_device_path(tmp_path):
    from gm2 import binary_converter as bc
    cases = json.load(open(os.path.join(ROOT, "tests", "golden", "converter.json")))["cases"]
    for case in cases:
        if "error" in case:
            continue
        mpath = tmp_path / f"{case['name']}.npy"
        np.save(mpath, np.asarray(case["masks"], dtype=case["mask_dtype"]))
        out = str(tmp_path / f"{case['name']}_ids.npy")
        ids = bc.masks_to_gene_lists(str(mpath), pd.Index(case["cols"]), out)
        assert [list(map(str, r)) for r in ids] == case["ids"]


def test_reconstruction_metrics_vs_sklearn():
    import sklearn.metrics
    from gm2.data import ResidentMatrix, StrainLoader
    from gm2.metrics import calculate_reconstruction_metrics
    G, H, L, N, BS = 900, 128, 16, 150, 64
    P, S = perturb_bn(*oracle_state(G, H, L, 80), seed=81)
    P["decoder.9.bias"] = torch.where(torch.arange(G) % 2 == 0, 2.5, -2.5)  # logits kept off the threshold
    X = synth_x(N, G, 82)
    m = to_model(P, S, G, H, L, native.GM2_BF16)  # the metrics forward is exact fp32 regardless
    torch.manual_seed(4)
    f1, acc, f1s, accs = calculate_reconstruction_metrics(m, StrainLoader(ResidentMatrix(X), None, BS), 0.5,
                                                         eps_rng="cpu")
    # oracle: the same per-batch eps (base seed draw, then one randn per batch), eval-mode forward
    torch.manual_seed(4)
    torch.empty((), dtype=torch.int64).random_()
    x = torch.tensor(X, dtype=torch.float32)
    recs, band = [], 0
    for s in range(0, N, BS):
        xb = x[s:s + BS]
        eps = torch.randn(xb.shape[0], L)
        r, mu, lv = O.forward(P, S, xb, eps, train=False)
        z = (mu + torch.exp(0.5 * lv) * eps)
        band += int((np.abs(O.decode_logits64(P, S, z).numpy()) <= 1e-4).sum())
        recs.append(r)
    assert band == 0, "fixture must be band-free for an exact comparison"
    rb = (torch.cat(recs) > 0.5).int().numpy()
    assert f1 == pytest.approx(sklearn.metrics.f1_score(X.flatten(), rb.flatten()), abs=1e-12)
    assert acc == pytest.approx(sklearn.metrics.accuracy_score(X.flatten(), rb.flatten()), abs=1e-12)
    ref_f1 = [sklearn.metrics.f1_score(a, b) for a, b in zip(rb, X.astype(int))]
    ref_acc = [sklearn.metrics.accuracy_score(a, b) for a, b in zip(rb, X.astype(int))]
    np.testing.assert_allclose(f1s, ref_f1, rtol=0, atol=1e-12)
    np.testing.assert_allclose(accs, ref_acc, rtol=0, atol=1e-12)
