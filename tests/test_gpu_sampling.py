"""`--mode sample` paths against the oracle:

  * sample_from_model (extras.py:192-203) with N > one decode chunk, so the chunked path of
    VAE.decode_mask runs and chunk boundaries are crossed (default 65,536-row chunks, and a
    smaller chunk that leaves a ragged last chunk);
  * focused sampling (main.py:351-370 as main.focused_samples): 100 default samples, the fewest-
    genes sample, its output-space nearest neighbour, z* + sigma * N(0, I) decoded;
  * sample -> train one epoch -> sample on the same model: the second sampling decodes with the
    trained weights (the fp32 decode shadows are re-derived after the bf16 optimizer steps).
  * the gated decode (GM2_OPT_SAMPLE_SPLIT, api.hip decode_split3) on a REFERENCE-produced fixture
    where it runs a mix of bf16x3 and exact-fp32 tiles (tests/golden/make_golden_sampling_split.py),
    with the certified-band fp64 recompute, and the exact path on the same fixture; every test that
    decodes asserts which path ran from the workspace counters (gm2.h GM2_STAT_*).
Bar: masks bit-exact to the oracle's fp32 decode outside the fp64 rounding band of each logit
(|logit64| <= 1e-3: counted, reported), probabilities rel 2e-5; on the reference-produced fixture
every bit (the band included) equals the reference's; with the band list forced to overflow every
bit equals the correctly rounded fp64 logit's decision.
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
    st0 = m.decode_stats()
    pm, _ = m.decode_bits(z.cuda(), chunk=chunk)
    st = _delta(st0, m.decode_stats())
    chunks = (N + chunk - 1) // chunk
    blocks = sum((min(chunk, N - s) + 255) // 256 for s in range(0, N, chunk)) * ((G + 255) // 256)
    print(f"decode path: {st}")
    # the default path: every chunk's output layer gated per tile; at these weights every tile's bound
    # admits a bf16 tier (single product or split; the bench reports which)
    assert st["split_decodes"] == chunks and st["exact_decodes"] == 0, st
    assert st["single_tiles"] + st["split_tiles"] == blocks and st["exact_tiles"] == 0, st
    assert st["band_overflow"] == 0 and st["band_elements"] > 0, st
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


def test_c3_trained_checkpoint_stratified_oracle():
    """Verdict r5 (the headline sample leg is never checked against the oracle): the bench's own
    sample-leg workload -- a v1 checkpoint (G = 55,039, hidden 512, latent 32) trained 10 epochs at lr
    1e-3, batch 4096, L1 0.01 on the synthetic 10,000-strain matrix (bench.py train_v1_checkpoint) --
    decodes 131,072 genomes (two 65,536-genome chunks) into packed masks on the default tiered path.
    Bars: the single tier carries most tiles (as in the bench line), every row's popcount equals the
    device's genome size, and 40 stratified rows (first and last of each chunk + 36 seeded random
    rows) decoded by the oracle from the same checkpoint are bit-exact outside |logit64| <= 1e-3 and
    equal to the fp64 decision wherever |logit64| > 2e-5."""
    from gm2.data import ResidentMatrix, StrainLoader, synthetic_pangenome
    from gm2.model import VAE
    from gm2.trainer import Adam, StepLR, create_v1_trainer
    G, H, L, N, chunk = 55039, 512, 32, 131072, 65536
    torch.manual_seed(11)
    m = VAE(G, H, L, precision=native.GM2_BF16)
    opt = Adam(m, lr=1e-3)
    tr = create_v1_trainer(m, opt, StepLR(opt), 10, 1.0, 0.01)
    mat = ResidentMatrix(synthetic_pangenome(10000, G, seed=4242))
    loader = StrainLoader(mat, None, 4096, shuffle=True)
    for ep in range(10):
        tr.train_epoch(loader, ep)
    del mat, loader
    m.eval()
    torch.manual_seed(0)
    z = torch.randn(N, L)
    st0 = m.decode_stats()
    pm, _ = m.decode_bits(z.cuda(), chunk=chunk)
    d = _delta(st0, m.decode_stats())
    print(f"trained v1 checkpoint (bench workload), {N} genomes: {d}")
    assert d["split_decodes"] == 2 and d["exact_decodes"] == 0, d
    assert d["single_tiles"] > d["split_tiles"] + d["exact_tiles"] / 4, d
    host = pm.bits.cpu().numpy()
    np.testing.assert_array_equal(np.bitwise_count(host).sum(axis=1, dtype=np.int64), pm.row_sizes())
    rng = np.random.Generator(np.random.PCG64(21))
    strata = sorted({0, chunk - 1, chunk, N - 1} | set(int(r) for r in rng.integers(0, N, size=36)))
    mask = np.unpackbits(host[strata], axis=1, count=G, bitorder="little").astype(bool)
    P = O.unflatten(m.params.detach().cpu().numpy(), G, H, L)
    S = {}
    for i, b in enumerate(O.BNS):
        S[b + ".running_mean"] = m.bn[i, 0].cpu()
        S[b + ".running_var"] = m.bn[i, 1].cpu()
        S[b + ".num_batches_tracked"] = torch.tensor(m.num_batches_tracked[i])
    zs = z[strata]
    assert _masks_ok(mask, P, S, zs) == 0
    l64 = O.decode_logits64(P, S, zs).numpy()
    dec64 = l64.astype(np.float32) > np.float32(8.940696716308594e-08)
    assert int(((mask != dec64) & (np.abs(l64) > 2e-5)).sum()) == 0


def _stats(m):
    st = m.decode_stats()
    return st["split_decodes"], st["exact_decodes"]


def _delta(before, after):
    return {k: after[k] - before[k] for k in after}


@pytest.mark.parametrize("G,H,L,N", [(2900, 512, 32, 5000), (1000, 128, 16, 777)])
def test_split3_decode_equals_exact_outside_its_bound(G, H, L, N):
    """GM2_OPT_SAMPLE_SPLIT (api.hip decode_split3): the output layer of the sampling decode as one
    bf16 GEMM over K' = 2H on the (hi | lo) splits, hi.hi + hi.lo + lo.hi per K-tile. The call took
    that path (workspace counter); its packed masks (split tiles + the certified band recomputed in
    fp64) differ from the exact-fp32 path's (option 0: no band recompute) only where the fp64 logit is
    within the exact path's own rounding of the threshold (|logit64| <= 2.5e-4 + 1e-7 here), both
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
    ws = m.workspace(native.GM2_F32, N)
    for split, single in ((0, 1), (1, 0), (1, 1)):  # exact; bf16x3 split; the single-product tier
        ws.set_option(native.OPT_SAMPLE_SPLIT, split)
        ws.set_option(native.OPT_SAMPLE_SINGLE, single)
        before = m.decode_stats()
        pm, _ = m.decode_bits(z)
        mask, _ = m.decode_mask(z)
        d = _delta(before, m.decode_stats())
        assert (d["split_decodes"], d["exact_decodes"]) == ((2, 0) if split else (0, 2)), d
        if split:  # (at these weights every tile admits the tier under test; a single-product tile whose
            # band overflows its slots is re-run -- and counted -- as split)
            assert (d["single_tiles"] > 0) if single else (d["single_tiles"] == 0 and d["split_tiles"] > 0), d
        bits = pm.bits.cpu().numpy()
        unpacked = np.unpackbits(bits, axis=1, bitorder="little")[:, :G]
        np.testing.assert_array_equal(unpacked, mask.cpu().numpy())
        # bits past G are zero (the tile past the row pitch wrote nothing there)
        assert not np.unpackbits(bits, axis=1, bitorder="little")[:, G:].any()
        out[split, single] = unpacked.astype(bool)
        assert _masks_ok(out[split, single], P, S, z) == 0
    ws.set_option(native.OPT_SAMPLE_SPLIT, 1)
    ws.set_option(native.OPT_SAMPLE_SINGLE, 1)
    l64 = O.decode_logits64(P, S, z).numpy()
    for key in ((1, 0), (1, 1)):
        diff = out[0, 1] != out[key]
        print(f"{key}: {int(diff.sum())} differences from the exact path, max |logit64| there "
              f"{float(np.abs(l64[diff]).max()) if diff.any() else 0.0:.3g}")
        assert np.all(np.abs(l64[diff]) <= 2.5e-4 + 1e-7)
    # both bf16 tiers decide every bit as the fp64 logit of the same fp32 activations does (outside
    # a tier's certified band from its own GEMM, inside it from the recompute): bit-identical
    np.testing.assert_array_equal(out[1, 0], out[1, 1])


def test_split3_decode_falls_back_when_the_bound_is_too_large():
    """Output weights x 200: the bound 4.62e-5 max||a|| max||w|| exceeds the gate (1e-3) on every tile, so the call runs the
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
        before = m.decode_stats()
        mask, _ = m.decode_mask(z)
        d = _delta(before, m.decode_stats())
        assert d["split_decodes"] == 0 and d["exact_decodes"] == 1 and d["split_tiles"] == 0 and d["single_tiles"] == 0, d
        if split:  # every tile of the gated decode ran exact fp32 (300 x 700: 3 x 6 tiles of 128)
            assert d["exact_tiles"] == 3 * 6, d
        res.append((mask.cpu().numpy().astype(bool), d))
    # the same fp32 kernel; the gated call also recomputed its certified band in fp64, which may
    # change only bits of band elements (and never more bits than it reports flipped)
    diff = int((res[0][0] != res[1][0]).sum())
    assert diff <= res[0][1]["band_flips"], (diff, res[0][1])
    assert _masks_ok(res[0][0], P, S, z) == 0 and _masks_ok(res[1][0], P, S, z) == 0
    # the exact tiles' band entries go straight to the shard lists: with one entry per shard, a tile
    # holding two or more overflows and is recomputed whole in fp64 -- the same masks
    ws = m.workspace(native.GM2_F32, N)
    ws.set_option(native.OPT_SAMPLE_SPLIT, 1)
    ws.set_option(native.OPT_SAMPLE_BAND_CAP, 1)
    before = m.decode_stats()
    mask, _ = m.decode_mask(z)
    d = _delta(before, m.decode_stats())
    ws.set_option(native.OPT_SAMPLE_BAND_CAP, 65536)
    print(f"band list capacity 1: {d}")
    assert (d["overflow_tiles"] > 0) == (d["band_overflow"] > 0), d
    np.testing.assert_array_equal(mask.cpu().numpy().astype(bool), res[0][0])


def _split_fixture():
    from golden_io import load
    g = load("sampling_split")
    G, H, L, N = [int(v) for v in g["dims"]]
    P, S = oracle_state(G, H, L, 0)
    for k in g.files:
        if k.startswith("sd/"):
            name = k[3:]
            (P if name in P else S)[name] = torch.tensor(g[k].astype(np.float32) if g[k].dtype == np.float16 else g[k])
    z = torch.tensor(g["z16"].astype(np.float32))
    ref = np.unpackbits(g["mask_bits"], axis=1, count=G, bitorder="little").astype(bool)
    near = np.zeros(N * G, dtype=np.float64) + np.inf  # fp64 logit where |logit| <= 2e-3, else inf
    near[g["near_idx"]] = g["near_logit64"]
    return g, (G, H, L, N), P, S, z, ref, near.reshape(N, G)


@pytest.mark.parametrize("single", [1, 0])
def test_split_fixture_gated_decode_matches_reference(single):
    """The gated sampling decode (default GM2_OPT_SAMPLE_SPLIT = 1) on a reference-produced fixture
    (tests/golden/make_golden_sampling_split.py: G 3,000, hidden 512, latent 32, 1,024 genomes; one
    genome block and one gene block scaled past the split bound): the tiles the fixture's fp64
    verdict admits run bf16x3, the rest exact fp32 (counted per path), logits in the certified band
    are recomputed in fp64. Bars, for the packed and the u8 output alike:
      * bit-exact to the reference's own masks outside |logit64| <= 1e-3;
      * every mask bit equals the correctly rounded fp64 logit's (float(logit64) > T) wherever
        |logit64| > 2e-5 -- the band recompute leaves only the hidden layers' fp32 noise;
      * counters: 2 x the fixture's split tiles, 2 x 4 x its exact 256-blocks (128-tiles), band
        elements found and recomputed, none past the list."""
    g, (G, H, L, N), P, S, z, ref, l64 = _split_fixture()
    m = to_model(P, S, G, H, L, native.GM2_F32)
    m.eval()
    m.workspace(native.GM2_F32, N).set_option(native.OPT_SAMPLE_SINGLE, single)
    verdict = g["split_verdict"].astype(bool)
    # the single-product tier's verdict from the same fp64 block bounds (the device's maxima come from
    # fp32 norms rounded up by 1e-4: blocks this close to the threshold are not asserted)
    ratio = g["split_bound"] * (7.83e-3 / 4.62e-5) / 0.25
    sv = (ratio <= 1.0) if single else np.zeros_like(verdict)
    ev = ~verdict & ~sv
    st0 = m.decode_stats()
    pm, _ = m.decode_bits(z)
    mask, _ = m.decode_mask(z)
    d = _delta(st0, m.decode_stats())
    print(f"decode path: {d}; fixture verdicts {int(sv.sum())} single / {int((verdict & ~sv).sum())} split / "
          f"{int(ev.sum())} exact blocks")
    assert d["split_decodes"] == 2 and d["exact_decodes"] == 0, d
    if not single or np.all(np.abs(np.log(ratio)) > 1e-3):
        # (a single-product tile whose band overflows its slots is re-run and counted as split)
        assert d["single_tiles"] <= 2 * int(sv.sum()), d
        assert d["single_tiles"] + d["split_tiles"] == 2 * int((sv | verdict).sum()), d
        assert d["exact_tiles"] == 2 * 4 * int(ev.sum()), d
    assert d["band_elements"] > 0 and d["band_overflow"] == 0, d
    bits = np.unpackbits(pm.bits.cpu().numpy(), axis=1, bitorder="little")
    assert not bits[:, G:].any()
    for got in (bits[:, :G].astype(bool), mask.cpu().numpy().astype(bool)):
        band = np.abs(l64) <= 1e-3
        bad = (got != ref) & ~band
        print(f"{int(((got != ref) & band).sum())} reference mismatches inside the 1e-3 band, {int(bad.sum())} outside")
        # (verdict r5: the reference's own masks, every bit -- inside the band too)
        np.testing.assert_array_equal(got, ref)
        # the fp64 decision: (float)logit64 > T
        dec64 = l64.astype(np.float32) > np.float32(8.940696716308594e-08)
        known = np.isfinite(l64) & (np.abs(l64) > 2e-5)
        assert int(((got != dec64) & known).sum()) == 0, int(((got != dec64) & known).sum())


def test_split_fixture_exact_path_matches_reference():
    """GM2_OPT_SAMPLE_SPLIT = 0 on the same reference fixture: the whole output layer in exact fp32
    (no tile gate, no band recompute; counted as an exact decode), bit-exact to the reference's masks
    outside |logit64| <= 1e-3."""
    g, (G, H, L, N), P, S, z, ref, l64 = _split_fixture()
    m = to_model(P, S, G, H, L, native.GM2_F32)
    m.eval()
    m.workspace(native.GM2_F32, N).set_option(native.OPT_SAMPLE_SPLIT, 0)
    st0 = m.decode_stats()
    mask, _ = m.decode_mask(z)
    d = _delta(st0, m.decode_stats())
    assert d["exact_decodes"] == 1 and d["split_decodes"] == 0 and d["split_tiles"] == 0 and d["band_elements"] == 0, d
    got = mask.cpu().numpy().astype(bool)
    band = np.abs(l64) <= 1e-3
    print(f"{int(((got != ref) & band).sum())} mismatches inside the 1e-3 band")
    assert int(((got != ref) & ~band).sum()) == 0
    np.testing.assert_array_equal(got, ref)  # (every bit, the band included)


def _hidden32(P, S, z):
    """the decoder's last hidden activations in fp32 (the oracle's eval-mode blocks)"""
    with torch.no_grad():
        h = z.float()
        for i in range(3):
            h = O._block(P, S, f"decoder.{3*i}", f"decoder.{3*i+1}", h, False)
    return h


@pytest.mark.parametrize("single,G,N", [(1, 1000, 600), (0, 1000, 600), (1, 777, 1), (1, 2999, 257)])
def test_band_overflow_recomputed_whole_blocks(single, G, N):
    """Verdict r5 "next" 1 / ADVICE r5: every logit sits inside the certified band, so the band list
    overflows, and no bit may be left as a bf16 tier decided it. The output weights are scaled to
    ~2.5e-14 and every gene's bias is the threshold T itself (0x33C00000): each logit is T + delta with
    |delta| of a few fp32 ulps of T (ulp 2^-47), far inside every tier's band (its 2^-20 T floor).
      * single tier on: every tile's band overflows its 256 slots, so each re-runs as bf16x3 in place
        (counted as split, ADVICE r5 gemm.hip:1408), whose band spills to the shard lists;
      * with the default shard capacity (64 x 65,536) k_band_fix recomputes every element; with
        GM2_OPT_SAMPLE_BAND_CAP = 64 the shards overflow and EVERY tile is recomputed whole in fp64
        by k_band_tile_fix (GM2_STAT_OVERFLOW_TILES);
    packed and u8 outputs, both capacities and both tier settings give the same bits, and those equal
    the correctly rounded fp64 logit's decision (float)(a . w + b) > T from the fp32 activations,
    except where the fp64 logit lies within 1e-20 of an fp32 rounding midpoint (the host's fp32
    hidden layers differ from the device's by ~1e-7 relative, i.e. ~1e-21 in these logits).
    Shapes: ragged genome and gene blocks (600 x 1000), one genome with a gene count that ends
    mid-word (777: the recomputed block's packed words past G stay zero), and 257 genomes (a second
    row block of one row) at 2,999 genes."""
    H, L = 128, 16
    P, S = perturb_bn(*oracle_state(G, H, L, 70), seed=71)
    T = np.float32(8.940696716308594e-08)
    assert T.view(np.uint32) == 0x33C00000
    P["decoder.9.weight"] = P["decoder.9.weight"] * 2.5e-14
    P["decoder.9.bias"] = torch.full((G,), float(T))
    m = to_model(P, S, G, H, L, native.GM2_F32)
    m.eval()
    z = torch.randn(N, L, generator=torch.Generator().manual_seed(72))
    tiles = ((N + 255) // 256) * ((G + 255) // 256)
    # logits per 256 x 256 block (every one is in the band)
    elems = [min(256, N - 256 * r) * min(256, G - 256 * c) for r in range((N + 255) // 256) for c in range((G + 255) // 256)]
    n_split = sum(1 for e in elems if e > 256) if single else tiles
    ws = m.workspace(native.GM2_F32, N)
    ws.set_option(native.OPT_SAMPLE_SINGLE, single)
    outs = []
    for cap in (65536, 64):
        ws.set_option(native.OPT_SAMPLE_BAND_CAP, cap)
        st0 = m.decode_stats()
        pm, _ = m.decode_bits(z)
        mask, _ = m.decode_mask(z)
        d = _delta(st0, m.decode_stats())
        print(f"single {single} cap {cap}: {d}")
        # both calls gated; every tile whose band (all its logits) exceeds the single tier's 256 slots
        # re-runs as bf16x3 (counted as split), the others stay single; a split tile's entries past its
        # 256 slots go to its shard, which overflows past `cap`
        assert d["split_decodes"] == 2 and d["exact_decodes"] == 0, d
        assert d["split_tiles"] == 2 * n_split and d["single_tiles"] == 2 * (tiles - n_split), d
        assert d["exact_tiles"] == 0, d
        assert d["band_elements"] >= 2 * N * G, d  # (pad genes are never in the band; every real logit is)
        n_ovf = sum(1 for e in elems if e > 256 + cap)  # (the tiles <= 64: one shard each, blockIdx % 64)
        if cap == 65536:
            assert d["band_overflow"] == 0 and d["overflow_tiles"] == 0, d
        else:
            assert (d["band_overflow"] > 0) == (n_ovf > 0) and d["overflow_tiles"] == 2 * n_ovf, d
        bits = np.unpackbits(pm.bits.cpu().numpy(), axis=1, bitorder="little")
        assert not bits[:, G:].any(), "pad bits beyond G must stay zero"
        np.testing.assert_array_equal(bits[:, :G], mask.cpu().numpy())
        outs.append(bits[:, :G].astype(bool))
    ws.set_option(native.OPT_SAMPLE_BAND_CAP, 65536)
    ws.set_option(native.OPT_SAMPLE_SINGLE, 1)
    np.testing.assert_array_equal(outs[0], outs[1])
    a = _hidden32(P, S, z).double().numpy()
    l64 = a @ P["decoder.9.weight"].double().numpy().T + np.float64(T)
    dec = l64.astype(np.float32) > T
    # distance to the nearest fp32 rounding midpoint around T (ulp(T) = 2^-47 on both sides here)
    ulp = 2.0 ** -47
    frac = (l64 - float(T)) / ulp
    ambiguous = np.abs(frac - np.round(frac - 0.5) - 0.5) * ulp < 1e-20
    print(f"{int(dec.sum())} of {dec.size} bits set; {int(ambiguous.sum())} ambiguous; max |logit - T| "
          f"{np.abs(l64 - float(T)).max():.3g} (band floor 2^-20 T = {2.0 ** -20 * float(T):.3g})")
    assert dec.any() and (N == 1 or not dec.all())
    assert int(((outs[0] != dec) & ~ambiguous).sum()) == 0


def test_trained_checkpoint_tiered_decode_vs_oracle():
    """Verdict r5 (the bench's sample leg is never checked against the oracle, and the C3 test decodes
    perturbed init weights, where every tile admits a bf16 tier): a v1 model (hidden 512, latent 32,
    abundance + L1) TRAINED 4 epochs at the reference's lr 1e-3 on a synthetic pan-genome matrix, as
    the bench trains its checkpoint, then 20,000 genomes through the default tiered decode. Bars: the
    tile counters show the tiers the trained weights admit (recorded), masks bit-exact to the
    oracle's fp32 decode of the same checkpoint outside |logit64| <= 1e-3, every bit equal to the
    correctly rounded fp64 logit's decision where |logit64| > 2e-5, and the tiered masks differ from
    the exact-fp32 path's (GM2_OPT_SAMPLE_SPLIT = 0, no band recompute) only where |logit64| <= 1e-3
    (that path's own fp32 rounding of the threshold)."""
    from gm2.data import ResidentMatrix, StrainLoader
    from gm2.trainer import Adam, StepLR, create_v1_trainer
    G, H, L, N = 5000, 512, 32, 20000
    torch.manual_seed(11)
    P0, S0 = oracle_state(G, H, L, 12)
    m = to_model(P0, S0, G, H, L, native.GM2_BF16)
    opt = Adam(m, lr=1e-3)
    tr = create_v1_trainer(m, opt, StepLR(opt), 4, 1.0, 0.01)
    loader = StrainLoader(ResidentMatrix(synth_x(4096, G, 13)), None, 512, shuffle=True)
    for ep in range(4):
        tr.train_epoch(loader, ep)
    m.eval()
    z = torch.randn(N, L, generator=torch.Generator().manual_seed(14))
    st0 = m.decode_stats()
    pm, _ = m.decode_bits(z)
    d = _delta(st0, m.decode_stats())
    print(f"trained v1 checkpoint, tiered decode: {d}")
    assert d["split_decodes"] + d["exact_decodes"] == 1, d
    got = np.unpackbits(pm.bits.cpu().numpy(), axis=1, count=G, bitorder="little").astype(bool)
    P = O.unflatten(m.params.detach().cpu().numpy(), G, H, L)
    S = {k: v.clone() for k, v in S0.items()}
    for i, b in enumerate(O.BNS):
        S[b + ".running_mean"] = m.bn[i, 0].cpu()
        S[b + ".running_var"] = m.bn[i, 1].cpu()
    assert _masks_ok(got, P, S, z) == 0
    l64 = O.decode_logits64(P, S, z).numpy()
    dec64 = l64.astype(np.float32) > np.float32(8.940696716308594e-08)
    known = np.abs(l64) > 2e-5
    assert int(((got != dec64) & known).sum()) == 0
    ws = m.workspace(native.GM2_F32, N)
    ws.set_option(native.OPT_SAMPLE_SPLIT, 0)
    ex, _ = m.decode_mask(z)
    ws.set_option(native.OPT_SAMPLE_SPLIT, 1)
    diff = ex.cpu().numpy().astype(bool) != got
    print(f"{int(diff.sum())} bits differ from the exact-fp32 path, max |logit64| there "
          f"{float(np.abs(l64[diff]).max()) if diff.any() else 0.0:.3g}")
    assert np.all(np.abs(l64[diff]) <= 1e-3)


def test_odd_latent_width_decodes_on_the_exact_path():
    """latent_dim = 1 (odd: the output weights start 4-B aligned in the parameter buffer,
    which the split kernels cannot read) -- the gated decode's preconditions fail before anything is
    launched and the call runs the exact path (counted as such) instead of failing."""
    G, H, L, N = 500, 128, 1, 700
    P, S = perturb_bn(*oracle_state(G, H, L, 95), seed=96)
    P["decoder.9.bias"] = torch.linspace(-1.0, 1.0, G)
    m = to_model(P, S, G, H, L, native.GM2_F32)
    m.eval()
    z = torch.randn(N, L, generator=torch.Generator().manual_seed(97))
    st0 = m.decode_stats()
    pm, _ = m.decode_bits(z)
    mask, _ = m.decode_mask(z)
    d = _delta(st0, m.decode_stats())
    assert d["exact_decodes"] == 2 and d["split_decodes"] == 0, d
    np.testing.assert_array_equal(np.unpackbits(pm.bits.cpu().numpy(), axis=1, count=G, bitorder="little"),
                                  mask.cpu().numpy())
    assert _masks_ok(mask.cpu().numpy(), P, S, z) == 0
