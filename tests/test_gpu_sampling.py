"""`--mode sample` paths against the oracle:

  * sample_from_model (extras.py:192-203) with N > one decode chunk, so the chunked path of
    VAE.decode_mask runs and chunk boundaries are crossed (default 65,536-row chunks, and a
    smaller chunk that leaves a ragged last chunk);
  * focused sampling (main.py:351-370 as main.focused_samples): 100 default samples, the fewest-
    genes sample, its output-space nearest neighbour, z* + sigma * N(0, I) decoded;
  * sample -> train one epoch -> sample on the same model: the second sampling decodes with the
    trained weights (the fp32 decode shadows are re-derived after the bf16 optimizer steps).
Bar: masks bit-exact to the oracle's fp32 decode outside the fp64 rounding band of each logit
(|logit64| <= 1e-3: counted, reported, not asserted), probabilities rel 2e-5.
"""
import numpy as np
import pytest
import torch

from gpu_helpers import oracle_state, perturb_bn, synth_x, to_model
from oracle import vae_oracle as O

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from gm2 import native


def _masks_ok(mask, P, S, z):
    ref = (O.sample_decode(P, S, z).numpy() > 0.5)
    l64 = O.decode_logits64(P, S, z).numpy()
    band = np.abs(l64) <= 1e-3
    bad = int(((np.asarray(mask).astype(bool) != ref) & ~band).sum())
    print(f"{int(band.sum())} band elements, {bad} mismatches outside the band")
    return bad


@pytest.mark.parametrize("N,chunk", [(70001, 65536), (70001, 30000)])
def test_sample_from_model_chunked(N, chunk):
    from gm2.extras import sample_from_model
    G, H, L = 257, 128, 16
    P, S = perturb_bn(*oracle_state(G, H, L, 40), seed=41)
    P["decoder.9.bias"] = torch.linspace(-1.5, 1.0, G)
    m = to_model(P, S, G, H, L, native.GM2_F32)
    m.eval()
    torch.manual_seed(123)
    binary, probs, z = sample_from_model(m, L, N, torch.device("cuda"), chunk=chunk)
    assert binary.shape == (N, G) and binary.dtype == np.float64 and z.shape == (N, L)
    zc = z.cpu()
    assert _masks_ok(binary, P, S, zc) == 0
    np.testing.assert_allclose(probs, O.sample_decode(P, S, zc).numpy(), rtol=2e-5, atol=2e-6)
    # z is the reference draw: torch.randn(N, L, device) from the seeded generator
    torch.manual_seed(123)
    np.testing.assert_array_equal(zc.numpy(), torch.randn(N, L, device="cuda").cpu().numpy())


def test_focused_sampling_matches_oracle():
    import main as cli
    G, H, L, N, sigma = 300, 128, 16, 500, 0.1
    P, S = perturb_bn(*oracle_state(G, H, L, 50), seed=51)
    P["decoder.9.bias"] = torch.linspace(-2.0, 0.5, G)
    m = to_model(P, S, G, H, L, native.GM2_F32)
    m.eval()
    dev = torch.device("cuda")
    torch.manual_seed(7)
    mask, z = cli.focused_samples(m, L, N, sigma, dev)
    # oracle: replay the two device draws, then the reference's selection and noise
    torch.manual_seed(7)
    z_temp = torch.randn(100, L, device=dev).cpu()
    noise = torch.randn(N, L, device=dev).cpu() * sigma
    p_temp = O.sample_decode(P, S, z_temp).numpy()
    b_temp = (p_temp > 0.5).astype(float)
    i_min = np.argmin(b_temp.sum(axis=1))
    closest = np.argmin(np.linalg.norm(p_temp - p_temp[i_min], axis=1))
    z_ref = z_temp[closest].unsqueeze(0) + noise
    np.testing.assert_allclose(z.cpu().numpy(), z_ref.numpy(), rtol=0, atol=1e-6)
    assert _masks_ok(mask.cpu().numpy(), P, S, z_ref) == 0


def test_sample_train_sample_uses_trained_weights():
    """decoding after training must use the updated weights, also when the fp32
    (sampling) workspace existed before a bf16 training epoch."""
    from gm2.data import ResidentMatrix, StrainLoader
    from gm2.trainer import Adam, StepLR, create_v0_trainer
    G, H, L = 300, 128, 16
    P, S = oracle_state(G, H, L, 60)
    m = to_model(P, S, G, H, L, native.GM2_BF16)
    z = torch.randn(64, L)
    m.eval()
    before, _ = m.decode_mask(z)
    opt = Adam(m, lr=1e-2)
    tr = create_v0_trainer(m, opt, StepLR(opt), 2, 1.0, 0.1, 1.0)
    x = synth_x(128, G, 61)
    tr.train_epoch(StrainLoader(ResidentMatrix(x), None, 64, shuffle=True), 0)
    m.eval()
    after, p_after = m.decode_mask(z, want_probs=True)
    Pn = O.unflatten(m.params.cpu().numpy(), G, H, L)
    Sn = {k: v.clone() for k, v in S.items()}
    for i, b in enumerate(O.BNS):
        Sn[b + ".running_mean"] = m.bn[i, 0].cpu()
        Sn[b + ".running_var"] = m.bn[i, 1].cpu()
    np.testing.assert_allclose(p_after.cpu().numpy(), O.sample_decode(Pn, Sn, z).numpy(), rtol=2e-5, atol=2e-6)
    assert not torch.equal(before, after)


def test_c3_million_genomes_properties_and_stratified_oracle():
    """C3 (BASELINE.json configs[2]): `--mode sample` of 1e6 genomes at v1 dims (G = 55,039,
    hidden 512, latent 32), z = torch.manual_seed(0); torch.randn(1e6, 32) on the host (SURVEY.md
    §8d), decoded in 65,536-genome chunks into packed masks on the device (VAE.decode_bits). Every
    row is checked by size-independent properties against a host recount of the packed rows that
    reached the host:
      * genome sizes (PackedMasks.row_sizes, the device popcount + scan) == host popcount per row;
      * the pad bit beyond G (bit 55,039 of the 6,880-byte row) is zero in every row;
      * essential-gene counts (PackedMasks.count_groups, a 300-gene table with 1-3 columns each,
        some negative) == the host's any-of-positions recount of every row;
    and a stratified subset -- the first and last genome of every chunk -- is decoded by the
    oracle: bit-exact outside the fp64 rounding band of each logit."""
    G, H, L, N, chunk = 55039, 512, 32, 1_000_000, 65536
    P, S = perturb_bn(*oracle_state(G, H, L, 60), seed=61)
    P["decoder.9.bias"] = torch.linspace(-2.0, 1.0, G)
    m = to_model(P, S, G, H, L, native.GM2_F32)
    m.eval()
    torch.manual_seed(0)
    z = torch.randn(N, L)
    pm, _ = m.decode_bits(z.cuda(), chunk=chunk)
    assert pm.n == N and pm.ld == native.packed_row_bytes(G) == 6880
    sizes = pm.row_sizes()
    rng = np.random.Generator(np.random.PCG64(7))
    ess = {f"e{i}": [int(p) for p in rng.integers(-G, G, size=int(rng.integers(1, 4)))] for i in range(300)}
    counts = pm.count_groups(ess)
    host = pm.bits.cpu().numpy()  # [N, 6880] packed rows
    del pm
    torch.cuda.empty_cache()
    assert int((host[:, G // 8] >> (G % 8)).max()) == 0, "pad bits beyond G must be zero"
    cols = [np.asarray(v) % G for v in ess.values()]
    for s in range(0, N, chunk):
        blk = host[s:s + chunk]
        np.testing.assert_array_equal(np.bitwise_count(blk).sum(axis=1, dtype=np.int64), sizes[s:s + chunk])
        recount = np.zeros(blk.shape[0], dtype=np.int64)
        for c in cols:
            recount += (((blk[:, c // 8] >> (c % 8)) & 1) != 0).any(axis=1)
        np.testing.assert_array_equal(recount, counts[s:s + chunk])
    strata = sorted({r for s in range(0, N, chunk) for r in (s, min(s + chunk, N) - 1)})
    zs = z[strata]
    mask = np.unpackbits(host[strata], axis=1, count=G, bitorder="little")
    print(f"mean genome size {sizes.mean():.1f} of {G}; mean essential count {counts.mean():.2f}; "
          f"{len(strata)} stratified rows")
    assert _masks_ok(mask, P, S, zs) == 0


def _stats(m):
    ws = m.workspace(native.GM2_F32, 1)
    return ws.stat(native.STAT_SPLIT_DECODES), ws.stat(native.STAT_EXACT_DECODES)


@pytest.mark.parametrize("G,H,L,N", [(2900, 512, 32, 5000), (1000, 128, 16, 777)])
def test_split3_decode_equals_exact_outside_its_bound(G, H, L, N):
    """GM2_OPT_SAMPLE_SPLIT (api.hip decode_split3): the output layer of the sampling decode as one
    bf16 GEMM over K' = 2H on the (hi | lo) splits, hi.hi + hi.lo + lo.hi per K-tile. The call took
    that path (workspace counter); its packed masks differ from the exact-fp32 path's only where the
    fp64 logit is within the path's stated bound of the threshold (|logit64| <= 2.5e-4 + 1e-7), both
    match the oracle outside the 1e-3 band, and the u8 and packed outputs agree -- two kernels on
    the split path: the packed one forms its bits by wave ballots from the MFMA fragments, the u8
    one through a byte image. G = 2900 leaves the last 256-gene tile past the packed row pitch (its
    stores must stop there); N = 5000 / 777 end in partial 256-genome tiles."""
    P, S = perturb_bn(*oracle_state(G, H, L, 80), seed=81)
    P["decoder.9.bias"] = torch.linspace(-1.0, 0.8, G)
    m = to_model(P, S, G, H, L, native.GM2_F32)
    m.eval()
    z = torch.randn(N, L, generator=torch.Generator().manual_seed(82))
    out = {}
    for split in (0, 1):
        m.workspace(native.GM2_F32, N).set_option(native.OPT_SAMPLE_SPLIT, split)
        before = _stats(m)
        pm, _ = m.decode_bits(z)
        mask, _ = m.decode_mask(z)
        after = _stats(m)
        assert (after[0] - before[0], after[1] - before[1]) == ((2, 0) if split else (0, 2)), (before, after)
        bits = pm.bits.cpu().numpy()
        unpacked = np.unpackbits(bits, axis=1, bitorder="little")[:, :G]
        np.testing.assert_array_equal(unpacked, mask.cpu().numpy())
        # bits past G are zero (the tile past the row pitch wrote nothing there)
        assert not np.unpackbits(bits, axis=1, bitorder="little")[:, G:].any()
        out[split] = unpacked.astype(bool)
        assert _masks_ok(out[split], P, S, z) == 0
    l64 = O.decode_logits64(P, S, z).numpy()
    diff = out[0] != out[1]
    print(f"{int(diff.sum())} split/exact differences, max |logit64| there "
          f"{float(np.abs(l64[diff]).max()) if diff.any() else 0.0:.3g}")
    assert np.all(np.abs(l64[diff]) <= 2.5e-4 + 1e-7)


def test_split3_decode_falls_back_when_the_bound_is_too_large():
    """Output weights x 200: the bound 4.62e-5 max||a|| max||w|| exceeds 2.5e-4, so the call runs the
    exact-fp32 output layer (workspace counter) and its masks are bit-identical to option 0's."""
    G, H, L, N = 700, 128, 16, 300
    P, S = perturb_bn(*oracle_state(G, H, L, 90), seed=91)
    P["decoder.9.weight"] = P["decoder.9.weight"] * 200.0
    m = to_model(P, S, G, H, L, native.GM2_F32)
    m.eval()
    z = torch.randn(N, L, generator=torch.Generator().manual_seed(92))
    res = []
    for split in (1, 0):
        m.workspace(native.GM2_F32, N).set_option(native.OPT_SAMPLE_SPLIT, split)
        before = _stats(m)
        mask, _ = m.decode_mask(z)
        after = _stats(m)
        assert after[0] == before[0] and after[1] == before[1] + 1
        res.append(mask.cpu())
    assert torch.equal(res[0], res[1])
