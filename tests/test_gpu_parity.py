"""GPU parity: libgm2 (HIP, gfx950) against the CPU oracle and the golden fixtures.

Tolerances (stated per test):
  * training step (both paths): the C2 method of tests/test_gpu_c2.py -- every gradient tensor's
    norm-wise error against the EXACT (fp64) oracle gradient is at most 3x the error of the
    reference arithmetic (the same math in fp32 on the device; for the bf16 path with the bf16 operand
    rounding emulated) + a floor (2e-4 / 1e-3); losses rel 1e-5 / 1e-4 against the
    sums of the same arithmetic; Adam abs 2e-7 from the GPU's own gradients.
  * sampled masks: bit-exact on every element outside the fp32 rounding band of its logit
    (|logit64| > 1e-3: counted and reported; band elements are reported, not asserted).
Pre-BN Linear biases have an exactly-zero true gradient (rounding noise on both sides) and are
compared with an absolute bound instead (SURVEY.md §7 'Hard parts').
"""
import numpy as np
import pytest
import torch

from golden_io import load
from gpu_helpers import oracle_state, perturb_bn, rel_err, scalars, synth_x, to_model
from oracle import vae_oracle as O

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from gm2 import native
    from gm2.data import ResidentMatrix


@pytest.fixture(params=[0, 1], ids=["loop2", "pingpong"])
def gemm_pp(request):
    """Both main loops of the 256x256 bf16 tiles (gm2_set_option GM2_OPT_GEMM_PP)."""
    old = native.get_option(native.OPT_GEMM_PP)
    native.set_option(native.OPT_GEMM_PP, request.param)
    yield request.param
    native.set_option(native.OPT_GEMM_PP, old)


@pytest.fixture(params=[0, 1], ids=["bnpass", "bnepi"])
def bn_epi(request):
    """BatchNorm statistics in the GEMM store epilogue, or the separate statistics pass
    (gm2_set_option GM2_OPT_BN_EPILOGUE)."""
    old = native.get_option(native.OPT_BN_EPILOGUE)
    native.set_option(native.OPT_BN_EPILOGUE, request.param)
    yield request.param
    native.set_option(native.OPT_BN_EPILOGUE, old)


@pytest.mark.parametrize("layout", ["nt", "nn", "tn"])
@pytest.mark.parametrize("prec", ["f32", "bf16"])
@pytest.mark.parametrize("M,N,K,splits", [(128, 128, 64, 1), (200, 300, 192, 1), (256, 1024, 1024, 1),
                                          (300, 256, 4096, 4), (1000, 130, 320, 1), (2048, 1024, 512, 1),
                                          # 256x256 ping-pong tiles: >= 256 tiles (nk = 1, 3), and the
                                          # long-K plan (big tiles + 8 split-K slices)
                                          (4000, 4096, 64, 1), (4096, 4000, 192, 1), (512, 512, 8192, -1)])
def test_gemm(prec, layout, M, N, K, splits, gemm_pp):
    """C = P.Q^T with each operand K-major ([rows][K]) or MN-major ([K][rows], read through
    ds_read_b64_tr_b16 / ds_read_b32): nt = both K-major (forward), nn = Q MN-major (input
    gradients), tn = both MN-major (weight gradients). fp32 accumulation of exact products."""
    g = torch.Generator().manual_seed(M * 7 + N * 13 + K)
    Mp, Np = -(-M // 128) * 128, -(-N // 128) * 128
    P = torch.randn(Mp, K, generator=g)
    Q = torch.randn(Np, K, generator=g)
    if prec == "bf16":
        P, Q = P.bfloat16().float(), Q.bfloat16().float()
    pk, qk = {"nt": (True, True), "nn": (True, False), "tn": (False, False)}[layout]
    Ps = P if pk else P.T.contiguous()
    Qs = Q if qk else Q.T.contiguous()
    dt = torch.bfloat16 if prec == "bf16" else torch.float32
    pr = native.GM2_BF16 if prec == "bf16" else native.GM2_F32
    Pd, Qd = Ps.to(dt).cuda(), Qs.to(dt).cuda()
    C = torch.full((M, N), float("nan"), device="cuda")
    slab = torch.empty(max(splits, 8) * M * N + 4, device="cuda") if splits != 1 else None
    native.gemm(pr, Pd, Ps.shape[1], Qd, Qs.shape[1], C, N, M, N, K, splits, slab, pk, qk)
    ref = (P[:M].double() @ Q[:N].double().T)
    err = (C.cpu().double() - ref).abs().max().item()
    scale = (P[:M].double().abs() @ Q[:N].double().abs().T).max().item()
    assert torch.isfinite(C).all()
    assert err <= 2e-6 * scale, (err, scale)


# The GEMMs of the v0 C2 step (B=4096, G=55,039 -> Gp=55,040, H=1024) at their real sizes, through
# gm2_gemm with the hot path's own tile / split plan (splits=-1); fp64 reference computed on the
# device from the same bf16 operands. (55040, 1024, 4096, tn) is the shape that faulted in the
# round-1 microbenchmark (gpurun_out/gemm_g1.log); (55039, ...) is the unpadded hot-path M.
@pytest.mark.parametrize("name,layout,M,N,K", [("dW9", "tn", 55040, 1024, 4096), ("dW9u", "tn", 55039, 1024, 4096),
                                               ("dWe0", "tn", 1024, 55040, 4096), ("dWe0u", "tn", 1024, 55039, 4096),
                                               ("dWe0nn", "nn", 1024, 55039, 4096), ("enc0", "nt", 4096, 1024, 55040),
                                               ("dA5", "nn", 4096, 1024, 55040), ("hid", "nt", 4096, 1024, 1024),
                                               ("hid_dX", "nn", 4096, 1024, 1024), ("hid_dW", "tn", 1024, 1024, 4096)])
def test_gemm_hot_shapes(name, layout, M, N, K, gemm_pp):
    """(dWe0u / dWe0nn: N = 55,039 = ldc, the [H][G] input-layer gradient whose rows are not 16-B
    aligned: row-shifted 16-B stores.)"""
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    Mp, Np = -(-M // 128) * 128, -(-N // 128) * 128
    pk, qk = {"nt": (True, True), "nn": (True, False), "tn": (False, False)}[layout]
    Ps = (torch.rand((Mp, K) if pk else (K, Mp), generator=g, device=dev) * 2 - 1).bfloat16()
    Qs = (torch.rand((Np, K) if qk else (K, Np), generator=g, device=dev) * 2 - 1).bfloat16()
    if pk:
        Ps[M:] = 0
    else:
        Ps[:, M:] = 0
    C = torch.full((M, N), float("nan"), device=dev)
    slab = torch.empty(8 * M * N + 4, device=dev)
    native.gemm(native.GM2_BF16, Ps, Ps.shape[1], Qs, Qs.shape[1], C, N, M, N, K, -1, slab, pk, qk)
    Pm = (Ps if pk else Ps.t())[:M].double()
    Qm = (Qs if qk else Qs.t())[:N].double()
    ref = Pm @ Qm.t()
    torch.cuda.synchronize()
    assert torch.isfinite(C).all()
    err = (C.double() - ref).abs().max().item()
    scale = (Pm.abs() @ Qm.abs().t()).max().item()
    assert err <= 2e-6 * scale, (name, err, scale)
    del Ps, Qs, C, slab, ref


@pytest.mark.parametrize("layout", ["nt", "nn", "tn"])
@pytest.mark.parametrize("prec", ["f32", "bf16"])
def test_gemm_asymmetric_layout(prec, layout):
    """A = I against an asymmetric B catches a transposed C/D map or tr-read map (guide §3)."""
    K = 128
    P = torch.eye(128)
    Q = (torch.arange(128 * K, dtype=torch.float32).reshape(128, K) % 97)
    pk, qk = {"nt": (True, True), "nn": (True, False), "tn": (False, False)}[layout]
    Ps = P if pk else P.T.contiguous()
    Qs = Q if qk else Q.T.contiguous()
    dt = torch.bfloat16 if prec == "bf16" else torch.float32
    pr = native.GM2_BF16 if prec == "bf16" else native.GM2_F32
    C = torch.empty(128, 128, device="cuda")
    native.gemm(pr, Ps.to(dt).cuda(), 128, Qs.to(dt).cuda(), 128, C, 128, 128, 128, K, 1, None, pk, qk)
    np.testing.assert_array_equal(C.cpu().numpy(), Q.T.numpy())


def _band_ok(mask_gpu, mask_ref, logit64):
    """Masks must agree on every element whose fp64 logit is outside the fp32 rounding band."""
    band = np.abs(logit64) <= 1e-3
    bad = (mask_gpu != mask_ref) & ~band
    print(f"mask band: {int(band.sum())} elements within 1e-3 of the threshold, "
          f"{int(((mask_gpu != mask_ref) & band).sum())} of them differ")
    return int(bad.sum()), int(band.sum())


def test_decode_masks_golden_bit_exact():
    g = load("sampling")
    tag = "p"  # H=256, L=32, G=300: preset-shaped fixture produced by the reference's VAE.decode
    G, H, L, N = [int(v) for v in g[f"{tag}_dims"]]
    P, S = oracle_state(G, H, L, 0)
    for k in g.files:
        if k.startswith(tag + "_sd/"):
            name = k[len(tag) + 4:]
            (P if name in P else S)[name] = torch.tensor(g[k])
    m = to_model(P, S, G, H, L, native.GM2_F32)
    st0 = m.decode_stats()
    mask, p = m.decode_mask(torch.tensor(g[f"{tag}_z"]), want_probs=True)
    st1 = m.decode_stats()
    # a probs request runs the whole output layer in exact fp32 (no tile gate): counted as such
    assert st1["exact_decodes"] - st0["exact_decodes"] == 1 and st1["split_tiles"] == st0["split_tiles"]
    bad, band = _band_ok(mask.cpu().numpy(), g[f"{tag}_mask"], g[f"{tag}_logit64"])
    assert bad == 0, (bad, band)
    # (verdict r5: every bit of the reference's own mask, inside the band too)
    np.testing.assert_array_equal(mask.cpu().numpy(), g[f"{tag}_mask"])
    np.testing.assert_allclose(p.cpu().numpy(), g[f"{tag}_p"], rtol=1e-5, atol=1e-6)
    # the default path (no probs): gated per 256 x 256 tile. The focused z (one latent point plus
    # 0.1 noise, main.py:351-370) keeps the activations small enough that both tiles (64 genomes x
    # 300 genes) pass the single-product bound: this reference vector pins the single bf16 kernel
    # (+ its band recompute) bit for bit, and with that tier off (GM2_OPT_SAMPLE_SINGLE = 0) the
    # bf16x3 kernel
    fm, _ = m.decode_mask(torch.tensor(g[f"{tag}_focused_z"]))
    st2 = m.decode_stats()
    d = {k: st2[k] - st1[k] for k in st2}
    print(f"focused decode path: {d}")
    assert d["split_decodes"] == 1 and d["single_tiles"] + d["split_tiles"] == 2 and d["exact_tiles"] == 0, d
    np.testing.assert_array_equal(fm.cpu().numpy(), g[f"{tag}_focused_mask"])
    ws = m.workspace(native.GM2_F32, 1)
    ws.set_option(native.OPT_SAMPLE_SINGLE, 0)
    fm, _ = m.decode_mask(torch.tensor(g[f"{tag}_focused_z"]))
    ws.set_option(native.OPT_SAMPLE_SINGLE, 1)
    st2b = m.decode_stats()
    d = {k: st2b[k] - st2[k] for k in st2b}
    print(f"focused decode path, single tier off: {d}")
    assert d["split_decodes"] == 1 and d["split_tiles"] == 2 and d["single_tiles"] == 0 and d["exact_tiles"] == 0, d
    np.testing.assert_array_equal(fm.cpu().numpy(), g[f"{tag}_focused_mask"])
    st2 = st2b
    # the fixture's main z without probs: the gated path, whatever each tile's verdict, bit-exact to
    # the reference outside the fp64 band
    gm, _ = m.decode_mask(torch.tensor(g[f"{tag}_z"]))
    st3 = m.decode_stats()
    d = {k: st3[k] - st2[k] for k in st3}
    print(f"main decode path: {d}")
    assert d["split_decodes"] + d["exact_decodes"] == 1 and d["single_tiles"] + d["split_tiles"] + d["exact_tiles"] > 0, d
    bad, band = _band_ok(gm.cpu().numpy(), g[f"{tag}_mask"], g[f"{tag}_logit64"])
    assert bad == 0, (bad, band)
    np.testing.assert_array_equal(gm.cpu().numpy(), g[f"{tag}_mask"])


@pytest.mark.parametrize("G,H,L,N", [(1000, 128, 16, 300), (3000, 512, 32, 2000), (2500, 1024, 64, 700)])
def test_decode_masks_vs_oracle(G, H, L, N):
    P, S = perturb_bn(*oracle_state(G, H, L, G + N), seed=5)
    P["decoder.9.bias"] = torch.linspace(-2.0, 1.0, G)
    torch.manual_seed(N)
    z = torch.randn(N, L)
    p_ref = O.sample_decode(P, S, z).numpy()
    l64 = O.decode_logits64(P, S, z).numpy()
    m = to_model(P, S, G, H, L, native.GM2_F32)
    mask, p = m.decode_mask(z, want_probs=True)
    bad, band = _band_ok(mask.cpu().numpy(), (p_ref > 0.5).astype(np.uint8), l64)
    assert bad == 0, f"{bad} mask bits differ outside the rounding band ({band} band elements)"
    np.testing.assert_allclose(p.cpu().numpy(), p_ref, rtol=2e-5, atol=2e-6)


def _prebn_bias(name):
    parts = name.split(".")
    return parts[0] in ("encoder", "decoder") and parts[1] in ("0", "3", "6") and parts[2] == "bias"


@pytest.mark.parametrize("prec", ["f32", "bf16"])
@pytest.mark.parametrize("G,H,L,B,wg,lam", [(300, 128, 16, 200, 0.0, 0.0), (517, 256, 32, 130, 0.55, 0.01),
                                            (1000, 128, 64, 64, 1.2, 0.01),
                                            # >= 128 256x256 output tiles: the big-tile recon kernel
                                            (8192, 256, 32, 1024, 0.55, 0.01)])
def test_train_step_vs_oracle(prec, G, H, L, B, wg, lam, gemm_pp, bn_epi):
    """One fused fwd+bwd (+clip+L1+Adam) against the oracle (trainer.py:109-120 semantics). The
    shapes cover both BatchNorm statistics routes under bn_epi=1: one-pass 128-row-tile GEMMs take
    them in the epilogue, the split-K input layer of the last shape keeps the separate pass.

    Gradient bar (the C2 method, tests/test_gpu_c2.py): per tensor, on the norm-wise relative error
    against EXACT (the oracle's explicit gradient in fp64 on the device),
        fro(libgm2) <= 3 * fro(reference arithmetic) + floor,
    where the reference arithmetic is the same math evaluated in fp32 on the device (torch fp32
    GEMMs), with the bf16 path's operand rounding for the bf16 path (manual_grads_emulated); floor
    2e-4 (f32) / 1e-3 (bf16)."""
    P, S = perturb_bn(*oracle_state(G, H, L, G + B), seed=9)
    X = synth_x(B, G, B)
    torch.manual_seed(1)
    eps = torch.randn(B, L)
    beta = 0.37
    pr = native.GM2_F32 if prec == "f32" else native.GM2_BF16
    m = to_model(P, S, G, H, L, pr)
    mat = ResidentMatrix(X)
    ws = m.workspace(pr, B)
    grads = torch.zeros_like(m.params)
    loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device="cuda")
    sc = scalars(beta=beta, wgamma=wg, lam=lam)
    ed = eps.cuda()
    native.train_fwd_bwd(ws, native.make_batch(mat.data, mat.ld, None, B, ed), m.params, grads, m.bn, sc, loss)
    native.grad_norm(ws, m.params, grads, sc, loss)
    torch.cuda.synchronize()
    # --- exact reference (fp64, device) and the reference arithmetic of this path
    dev = torch.device("cuda")
    x = torch.tensor(X, dtype=torch.float32)
    Pd = {k: v.to(dev) for k, v in P.items()}
    Sd = {k: v.to(dev) for k, v in S.items()}
    exact, sums = O.manual_grads_emulated(Pd, Sd, x.to(dev), ed, beta, wg)
    # the reference arithmetic: the same math in fp32 (+ the bf16 path's operand rounding)
    ref, sums_r = O.manual_grads_emulated(Pd, Sd, x.to(dev), ed, beta, wg,
                                          operand_round=O.bf16_round if prec == "bf16" else None,
                                          dtype=torch.float32)
    if prec == "bf16":
        sums = sums_r  # the loss of the bf16 arithmetic (rounded operands)
    lt = loss.cpu().numpy()
    rtol_loss = 1e-5 if prec == "f32" else 1e-4
    assert abs(lt[0] - sums[0]) <= rtol_loss * abs(sums[0]), (lt[0], sums[0])
    assert abs(lt[1] - sums[1]) <= rtol_loss * abs(sums[1]), (lt[1], sums[1])
    assert abs(lt[2] - sums[2]) <= 1e-4 * abs(sums[2]) + 1e-3 * B * L * (1 if prec == "bf16" else 0.01)
    off = m.offsets
    fails = []
    floor = 2e-4 if prec == "f32" else 1e-3
    for i, (name, shp) in enumerate(m.specs):
        got = grads[off[i]:off[i + 1]].cpu().double().numpy()
        ex = exact[name].reshape(-1).cpu().double().numpy()
        if _prebn_bias(name):
            scale = max(float(np.abs(exact[name.replace("bias", "weight")].cpu().numpy()).max()), 1e-12)
            if np.abs(got).max() > (1e-3 if prec == "f32" else 2e-2) * scale:
                fails.append(f"{name}: |g|max {np.abs(got).max():.3g} vs weight scale {scale:.3g}")
            continue
        r = ref[name].reshape(-1).cpu().double().numpy()
        nrm = max(float(np.linalg.norm(ex)), 1e-30)
        f_gpu = float(np.linalg.norm(got - ex)) / nrm
        f_ref = float(np.linalg.norm(r - ex)) / nrm
        msg = f"{name}: libgm2 {prec} vs exact fro {f_gpu:.3g}; reference arithmetic fro {f_ref:.3g}"
        print(msg)
        if not f_gpu <= 3 * f_ref + floor:
            fails.append(msg)
    assert not fails, "\n".join(fails)
    # BN running statistics (train-mode update, momentum 0.1, unbiased var) against the fp64 forward
    S2 = {k: v.double().clone() for k, v in S.items()}
    O.forward({k: v.double() for k, v in P.items()}, S2, x.double(), eps.double(), train=True)
    bn = m.bn.cpu().numpy()
    for i, b in enumerate(O.BNS):
        np.testing.assert_allclose(bn[i, 0], S2[b + ".running_mean"].numpy(), rtol=1e-3 if prec == "bf16" else 2e-5,
                                   atol=2e-3 if prec == "bf16" else 2e-6)
        np.testing.assert_allclose(bn[i, 1], S2[b + ".running_var"].numpy(), rtol=1e-2 if prec == "bf16" else 2e-5,
                                   atol=1e-3 if prec == "bf16" else 2e-6)
    # L1 statistic and clip norm
    l1 = sum(v.double().abs().sum().item() for v in P.values())
    if lam:
        assert abs(lt[3] - l1) <= 1e-6 * l1
    else:
        assert lt[3] == 0.0  # no L1 component: the clip pass reads gradients only
    tot = torch.cat([(exact[n].cpu().double() + lam * torch.sign(P[n]).double()).reshape(-1) for n in P])
    norm = tot.norm().item()
    assert abs(lt[4] - norm) <= (1e-4 if prec == "f32" else 3e-2) * norm
    # Adam step on the clipped grads: compare with the oracle's update from the GPU's own grads
    ge = grads.cpu()
    p0 = m.params.cpu()
    mom = torch.zeros_like(m.params)
    vel = torch.zeros_like(m.params)
    native.adam_step(ws, m.params, grads, mom, vel, sc)
    torch.cuda.synchronize()
    coef = min(1.0, 1.0 / (lt[4] + 1e-6))
    gg = (ge + lam * torch.sign(p0)) * np.float32(coef)
    st = O.AdamState(lr=1e-3)
    Pf = {"p": p0.clone()}
    O.adam_step(Pf, {"p": gg}, st)
    np.testing.assert_allclose(m.params.cpu().numpy(), Pf["p"].numpy(), rtol=0, atol=2e-7)
    np.testing.assert_allclose(mom.cpu().numpy(), st.m["p"].numpy(), rtol=1e-6, atol=1e-12)


@pytest.mark.parametrize("prec", ["f32", "bf16"])
def test_eval_forward_and_encode(prec):
    G, H, L, B = 700, 256, 32, 150
    P, S = perturb_bn(*oracle_state(G, H, L, 3), seed=4)
    X = synth_x(B, G, 2)
    torch.manual_seed(2)
    eps = torch.randn(B, L)
    pr = native.GM2_F32 if prec == "f32" else native.GM2_BF16
    m = to_model(P, S, G, H, L, pr)
    mat = ResidentMatrix(X)
    ws = m.workspace(pr, B)
    loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device="cuda")
    native.eval_forward(ws, native.make_batch(mat.data, mat.ld, None, B, eps.cuda()), m.params, m.bn,
                        scalars(beta=0.2), loss)
    x = torch.tensor(X, dtype=torch.float32)
    recon, mu, lv = O.forward(P, S, x, eps, train=False)
    bce = torch.nn.functional.binary_cross_entropy(recon, x, reduction="sum").item()
    lt = loss.cpu().numpy()
    assert abs(lt[0] - bce) <= (3e-5 if prec == "f32" else 3e-3) * bce
    mu_g, lv_g = m.encode(mat)
    assert rel_err(mu_g.cpu().numpy(), mu.detach().numpy()) <= (1e-5 if prec == "f32" else 2e-2)
    assert rel_err(lv_g.cpu().numpy(), lv.detach().numpy()) <= (1e-5 if prec == "f32" else 2e-2)
    # eval mode must not touch the running statistics
    np.testing.assert_array_equal(m.bn[0, 0].cpu().numpy(), S["encoder.1.running_mean"].numpy())


def test_gather_rows_matches_indexing():
    G, H, L, B = 333, 128, 16, 77
    X = synth_x(500, G, 6)
    rows = torch.randint(0, 500, (B,), generator=torch.Generator().manual_seed(0))
    P, S = oracle_state(G, H, L, 0)
    m = to_model(P, S, G, H, L, native.GM2_F32)
    mat = ResidentMatrix(X)
    mu_all, _ = m.encode(ResidentMatrix(X[rows.numpy()]))
    ws = m.workspace(native.GM2_F32, B)
    mu = torch.empty(B, L, device="cuda")
    native.encode(ws, native.make_batch(mat.data, mat.ld, rows.to(torch.int32).cuda(), B, None), m.params, m.bn,
                  mu, None)
    np.testing.assert_array_equal(mu.cpu().numpy(), mu_all.cpu().numpy())


@pytest.mark.parametrize("prec", ["f32", "bf16"])
@pytest.mark.parametrize("G,H,L,B", [(517, 128, 16, 130), (8192, 256, 32, 1024)])
def test_staged_next_batch_bit_identical(prec, G, H, L, B):
    """gm2_batch.next: a training call gathers the next batch's rows into the second input slot under
    its own tail. Steps that use a staged batch must be bit-identical to steps that gather their
    own rows, including a staged batch that is then NOT used (a different batch follows), a ragged
    last batch, and an eval call between two training calls (which discards the stage)."""
    P, S = perturb_bn(*oracle_state(G, H, L, 3 * G + B), seed=4)
    X = synth_x(3 * B, G, 11)
    pr = native.GM2_F32 if prec == "f32" else native.GM2_BF16
    gen = torch.Generator().manual_seed(5)
    sizes = [B, B, B - 37, B, B]
    rows = [torch.randperm(3 * B, generator=gen)[:n].to(torch.int32).cuda() for n in sizes]
    other = torch.randperm(3 * B, generator=gen)[:B].to(torch.int32).cuda()
    eps = [torch.randn(n, L, generator=gen).cuda() for n in sizes]
    sc = scalars(beta=0.37, wgamma=0.55, lam=0.0)

    def run(staged):
        m = to_model(P, S, G, H, L, pr)
        mat = ResidentMatrix(X)
        ws = m.workspace(pr, B)
        out = []
        for i, n in enumerate(sizes):
            nxt = None
            if staged and i + 1 < len(sizes):
                # step 1 stages `other` but step 2 is given its own rows (a miss); step 2 -> 3 is then
                # interrupted by an eval call
                nr = other if i == 1 else rows[i + 1]
                nxt = native.make_batch(mat.data, mat.ld, nr, B if i == 1 else sizes[i + 1], None)
            grads = torch.zeros_like(m.params)
            loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device="cuda")
            native.train_fwd_bwd(ws, native.make_batch(mat.data, mat.ld, rows[i], n, eps[i], next=nxt), m.params,
                                 grads, m.bn, sc, loss)
            if i == 3:
                el = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device="cuda")
                native.eval_forward(ws, native.make_batch(mat.data, mat.ld, other, B, eps[0]), m.params, m.bn, sc, el)
                out.append(el.cpu())
            out.append(grads.cpu())
            out.append(loss.cpu())
        torch.cuda.synchronize()
        return out

    a, b = run(False), run(True)
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize("G,B", [(16384, 256), (16500, 300)])
def test_input_layer_quarter_launches_bit_identical(G, B):
    """GM2_OPT_INPUT_CHUNKS = 4: the input-layer weight gradient as four row-quarter launches (one per
    gradient bucket 2..5, for the data-parallel exchange) gives the same gradient bit for bit as the
    single launch; the bucket bounds tile encoder.0.weight by quarters of its rows."""
    H, L = 1024, 32
    P, S = perturb_bn(*oracle_state(G, H, L, G + B), seed=12)
    X = synth_x(B, G, 13)
    eps = torch.randn(B, L, generator=torch.Generator().manual_seed(3)).cuda()
    sc = scalars(beta=0.37, wgamma=0.0, lam=0.0)
    old = native.get_option(native.OPT_INPUT_CHUNKS)
    outs = []
    try:
        for chunks in (1, 4):
            native.set_option(native.OPT_INPUT_CHUNKS, chunks)
            m = to_model(P, S, G, H, L, native.GM2_BF16)
            mat = ResidentMatrix(X)
            ws = m.workspace(native.GM2_BF16, B)
            grads = torch.zeros_like(m.params)
            loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device="cuda")
            native.train_fwd_bwd(ws, native.make_batch(mat.data, mat.ld, None, B, eps), m.params, grads, m.bn, sc,
                                 loss)
            native.grad_norm(ws, m.params, grads, sc, loss)
            torch.cuda.synchronize()
            outs.append((grads.cpu(), loss.cpu()))
    finally:
        native.set_option(native.OPT_INPUT_CHUNKS, old)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])  # incl. the clip norm (statistics re-read when chunked)
    bounds = native.grad_bucket_bounds(native.dims(G, H, L, B))
    assert len(bounds) == native.GRAD_BUCKETS == 6
    assert [b for b in bounds[2:]] == [(q * H // 4 * G, (q + 1) * H // 4 * G) for q in range(4)]


@pytest.mark.parametrize("G", [20480, 20000])
def test_capped_grid_bit_identical(G):
    """GM2_OPT_GRID_CAP: the output-layer weight-gradient GEMM on a capped grid (workgroups loop over
    tiles: 320 tiles -> 160 workgroups x 2 at G = 20480), the input-layer one and the output-layer
    loss GEMM (320 genes x strains tiles) give the same gradient, loss record and clip statistics bit
    for bit as one workgroup per tile; G = 20000 is padded to 20,224 = 79 x 256 in the bf16 workspace
    and takes the same 256-tile plans."""
    H, L, B = 1024, 32, 1024
    P, S = perturb_bn(*oracle_state(G, H, L, G + B), seed=31)
    X = synth_x(B, G, 32)
    eps = torch.randn(B, L, generator=torch.Generator().manual_seed(33)).cuda()
    sc = scalars(beta=0.37, wgamma=0.55, lam=0.0)
    sc[native.S_NORM_AHEAD] = 1.0
    old = native.get_option(native.OPT_GRID_CAP)
    outs = []
    try:
        for cap in (0, 7):
            native.set_option(native.OPT_GRID_CAP, cap)
            m = to_model(P, S, G, H, L, native.GM2_BF16)
            mat = ResidentMatrix(X)
            ws = m.workspace(native.GM2_BF16, B)
            grads = torch.zeros_like(m.params)
            loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device="cuda")
            native.train_fwd_bwd(ws, native.make_batch(mat.data, mat.ld, None, B, eps), m.params, grads, m.bn, sc,
                                 loss)
            native.grad_norm(ws, m.params, grads, sc, loss)
            torch.cuda.synchronize()
            outs.append((grads.cpu(), loss.cpu()))
    finally:
        native.set_option(native.OPT_GRID_CAP, old)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("G", [20480, 16500])
def test_backward_schedule_options_bit_identical(G):
    """GM2_OPT_INPUT_CHUNKS (the input-layer weight gradient as four row-quarter launches) and
    GM2_OPT_SIDE_STREAM = 0 (every weight gradient on the caller's stream) only reorder launches:
    gradients, loss record and clip statistics are bit-identical to the default schedule."""
    H, L, B = 1024, 32, 1024
    P, S = perturb_bn(*oracle_state(G, H, L, G + 7), seed=41)
    X = synth_x(B, G, 42)
    eps = torch.randn(B, L, generator=torch.Generator().manual_seed(43)).cuda()
    sc = scalars(beta=0.37, wgamma=0.55, lam=0.0)
    sc[native.S_NORM_AHEAD] = 1.0
    outs = []
    for side, chunks in ((1, 1), (1, 4), (0, 1), (0, 4)):
        m = to_model(P, S, G, H, L, native.GM2_BF16)
        mat = ResidentMatrix(X)
        ws = m.workspace(native.GM2_BF16, B)
        ws.set_option(native.OPT_SIDE_STREAM, side)
        ws.set_option(native.OPT_INPUT_CHUNKS, chunks)
        grads = torch.zeros_like(m.params)
        loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device="cuda")
        native.train_fwd_bwd(ws, native.make_batch(mat.data, mat.ld, None, B, eps), m.params, grads, m.bn, sc, loss)
        native.grad_norm(ws, m.params, grads, sc, loss)
        torch.cuda.synchronize()
        outs.append((grads.cpu(), loss.cpu()))
    for o in outs[1:]:
        assert torch.equal(outs[0][0], o[0])
        assert torch.equal(outs[0][1][:3], o[1][:3])
    # the clip statistics: from the GEMM epilogues (one input-layer launch) or the re-reading pass
    for o in outs[1:]:
        assert float(o[1][4]) == pytest.approx(float(outs[0][1][4]), rel=1e-6)


@pytest.mark.parametrize("G,B,rows_none", [(16384, 1024, False), (20000, 1000, False), (16384, 1024, True)])
def test_zero_copy_rows_bit_identical(G, B, rows_none):
    """gm2_batch.resident (ABI 4): a bf16 training call reads its rows in place from the resident
    operands (gm2_resident_build) -- the input-layer GEMM's rows, the input-layer weight gradient's
    k-rows and the loss epilogue's target bits through the batch's row indices -- instead of
    gathering them. To prove the in-place path ran, the batch's u8 `data` is a DIFFERENT matrix (all
    zeros) than the one the resident operands were built from: three steps (fwd+bwd, clip
    statistics, Adam) must still equal, bit for bit, the gathering run on the resident's own matrix,
    including a ragged batch (1000 rows: pad rows read the zero row) and rows = NULL (first n rows)."""
    H, L = 1024, 32
    S = 2 * B + 5
    P, Sb = perturb_bn(*oracle_state(G, H, L, G + B + 3), seed=61)
    X = synth_x(S, G, 62)
    gen = torch.Generator().manual_seed(63)
    rows = [None if rows_none else torch.randperm(S, generator=gen)[:B].to(torch.int32).cuda() for _ in range(3)]
    eps = [torch.randn(B, L, generator=gen).cuda() for _ in range(3)]
    outs = []
    for zero_copy in (False, True):
        m = to_model(P, Sb, G, H, L, native.GM2_BF16)
        mat = ResidentMatrix(X)
        res = mat.operands(native.GM2_BF16) if zero_copy else None
        data = torch.zeros_like(mat.data) if zero_copy else mat.data
        ws = m.workspace(native.GM2_BF16, B)
        grads = torch.zeros_like(m.params)
        mom, vel = torch.zeros_like(m.params), torch.zeros_like(m.params)
        out = []
        for i in range(3):
            sc = scalars(beta=0.37, wgamma=0.55, lam=0.01, step=i + 1)
            sc[native.S_NORM_AHEAD] = 1.0
            loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device="cuda")
            batch = native.make_batch(data, mat.ld, rows[i], B, eps[i], resident=res)
            native.train_fwd_bwd(ws, batch, m.params, grads, m.bn, sc, loss)
            native.grad_norm(ws, m.params, grads, sc, loss)
            out += [grads.clone(), loss.clone()]
            native.adam_step(ws, m.params, grads, mom, vel, sc)
        ws.join()
        torch.cuda.synchronize()
        outs.append(out + [m.params.clone(), m.bn.clone(), mom.clone(), vel.clone()])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_grad_bucket_events_off_bit_identical():
    """GM2_OPT_GRAD_BUCKETS = 0 (one process, no exchange): the backward records no bucket events --
    same gradients and loss record bit for bit -- and gm2_wait_grad_bucket then fails loudly; with
    the default every bucket can be waited on (buckets 2..5 of the one-launch input layer share one
    event)."""
    G, H, L, B = 16500, 1024, 32, 1024
    P, S = perturb_bn(*oracle_state(G, H, L, G + 9), seed=81)
    X = synth_x(B, G, 82)
    eps = torch.randn(B, L, generator=torch.Generator().manual_seed(83)).cuda()
    sc = scalars(beta=0.37, wgamma=0.55, lam=0.0)
    sc[native.S_NORM_AHEAD] = 1.0
    outs = []
    for rec in (1, 0):
        m = to_model(P, S, G, H, L, native.GM2_BF16)
        mat = ResidentMatrix(X)
        ws = m.workspace(native.GM2_BF16, B)
        ws.set_option(native.OPT_GRAD_BUCKETS, rec)
        grads = torch.zeros_like(m.params)
        loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device="cuda")
        native.train_fwd_bwd(ws, native.make_batch(mat.data, mat.ld, None, B, eps), m.params, grads, m.bn, sc, loss)
        s = torch.cuda.Stream()
        if rec:
            for b in range(native.GRAD_BUCKETS):
                native.wait_grad_bucket(ws, b, s)
        else:
            with pytest.raises(RuntimeError, match="GM2_OPT_GRAD_BUCKETS"):
                native.wait_grad_bucket(ws, 2, s)
        native.grad_norm(ws, m.params, grads, sc, loss)
        torch.cuda.synchronize()
        outs.append((grads.cpu(), loss.cpu()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


def test_resident_operands_match_the_matrix():
    """gm2_resident_build: rows < S are the 0/1 matrix in bf16 / f32 with zero pad columns up to
    ld = roundup(G, 256), row S (and the allocation's tail) zero, and the packed bits match numpy
    packbits(bitorder='little') of each row."""
    G, S = 1000, 77
    X = synth_x(S, G, 64)
    mat = ResidentMatrix(X)
    for prec, dt in ((native.GM2_BF16, torch.bfloat16), (native.GM2_F32, torch.float32)):
        r = mat.operands(prec)
        assert r.ld == 1024 and r.rows_t.dtype == dt and r.rows_t.shape[0] >= S + 1
        full = r.rows_t.float().cpu().numpy()
        np.testing.assert_array_equal(full[:S, :G], X.astype(np.float32))
        assert not full[:S, G:].any() and not full[S:].any()
        bits = r.bits.cpu().numpy().view(np.uint8)
        want = np.packbits(X.astype(np.uint8), axis=1, bitorder="little")
        np.testing.assert_array_equal(bits[:S, :want.shape[1]], want)
        assert not bits[:S, want.shape[1]:].any() and not bits[S:].any()


def test_two_workspaces_keep_their_own_options_and_state():
    """ABI 3: tuning options, side stream, gradient-bucket events and the staged input slot belong to
    the workspace. Two models trained interleaved in one process, one with the ping-pong main loop,
    capped grids and four input-layer launches, the other with the two-stage loop, no capped grid
    and one launch, each read back their own options, and each step is bit-identical to the same
    step run with that model alone; the process defaults are untouched."""
    G, H, L, B = 16384, 1024, 32, 512
    P, S = perturb_bn(*oracle_state(G, H, L, 91), seed=92)
    X = synth_x(2 * B, G, 93)
    gen = torch.Generator().manual_seed(94)
    rows = [torch.randperm(2 * B, generator=gen)[:B].to(torch.int32).cuda() for _ in range(3)]
    eps = [torch.randn(B, L, generator=gen).cuda() for _ in range(3)]
    sc = scalars(beta=0.37, wgamma=0.55, lam=0.01)
    defaults = {k: native.get_option(k) for k in (native.OPT_GEMM_PP, native.OPT_GRID_CAP, native.OPT_INPUT_CHUNKS)}
    cfg = {"a": {native.OPT_GEMM_PP: 1, native.OPT_GRID_CAP: 7, native.OPT_INPUT_CHUNKS: 4},
           "b": {native.OPT_GEMM_PP: 0, native.OPT_GRID_CAP: 0, native.OPT_INPUT_CHUNKS: 1}}

    def setup(tag):
        m = to_model(P, S, G, H, L, native.GM2_BF16)
        ws = m.workspace(native.GM2_BF16, B)
        for k, v in cfg[tag].items():
            ws.set_option(k, v)
        return m, ws, ResidentMatrix(X)

    def step(state, i):
        m, ws, mat = state
        grads = torch.zeros_like(m.params)
        loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device="cuda")
        native.train_fwd_bwd(ws, native.make_batch(mat.data, mat.ld, rows[i], B, eps[i]), m.params, grads, m.bn, sc,
                             loss)
        stream = torch.cuda.Stream()
        for b in range(native.GRAD_BUCKETS):
            native.wait_grad_bucket(ws, b, stream)  # this workspace's own bucket events
        torch.cuda.current_stream().wait_stream(stream)
        native.grad_norm(ws, m.params, grads, sc, loss)
        return grads.cpu(), loss.cpu(), m.bn.cpu()

    alone = {}
    for tag in ("a", "b"):
        st = setup(tag)
        alone[tag] = [step(st, i) for i in range(3)]
    sa, sb = setup("a"), setup("b")
    inter = {"a": [], "b": []}
    for i in range(3):
        inter["a"].append(step(sa, i))
        inter["b"].append(step(sb, i))
    torch.cuda.synchronize()
    for tag, st in (("a", sa), ("b", sb)):
        for k, v in cfg[tag].items():
            assert st[1].get_option(k) == v
        for x, y in zip(alone[tag], inter[tag]):
            for u, w in zip(x, y):
                assert torch.equal(u, w)
    assert {k: native.get_option(k) for k in defaults} == defaults


@pytest.mark.parametrize("prec", ["f32", "bf16"])
def test_deferred_output_adam_bit_identical(prec):
    """GM2_OPT_DEFER_OUTPUT_ADAM = n: the output layer's Adam update of step i is queued (with a copy
    of step i's scalar block, whose tensor is gone by then) and launched on the workspace's side
    stream after step i+1's input-layer GEMM on n workgroups per CU, joined right before step i+1's
    output layer. Four steps (fwd+bwd, clip statistics, Adam) give parameters, moments, gradients,
    losses and BN statistics bit-identical to the in-step update, with n = 1 and 3 and with an
    explicit Workspace.join() after a step (the queued update then runs on the caller's stream); a
    read of the parameters after Workspace.join() sees the final update."""
    G, H, L, B = 3000, 256, 32, 512
    P, S = perturb_bn(*oracle_state(G, H, L, 71), seed=72)
    X = synth_x(2 * B, G, 73)
    gen = torch.Generator().manual_seed(74)
    rows = [torch.randperm(2 * B, generator=gen)[:B].to(torch.int32).cuda() for _ in range(4)]
    eps = [torch.randn(B, L, generator=gen).cuda() for _ in range(4)]
    pr = native.GM2_F32 if prec == "f32" else native.GM2_BF16
    outs = []
    for defer, join_after in ((0, None), (1, None), (3, None), (2, 1)):
        m = to_model(P, S, G, H, L, pr)
        mat = ResidentMatrix(X)
        ws = m.workspace(pr, B)
        ws.set_option(native.OPT_DEFER_OUTPUT_ADAM, defer)
        grads = torch.zeros_like(m.params)
        mom, vel = torch.zeros_like(m.params), torch.zeros_like(m.params)
        losses = []
        for i in range(4):
            sc = scalars(beta=0.37, wgamma=0.55, lam=0.01, step=i + 1)
            loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device="cuda")
            native.train_fwd_bwd(ws, native.make_batch(mat.data, mat.ld, rows[i], B, eps[i]), m.params, grads, m.bn,
                                 sc, loss)
            native.grad_norm(ws, m.params, grads, sc, loss)
            native.adam_step(ws, m.params, grads, mom, vel, sc)
            del sc
            if i == join_after:
                ws.join()
            losses.append(loss)
        ws.join()
        outs.append([m.params.clone(), mom.clone(), vel.clone(), grads.clone(), m.bn.clone()] + losses)
    torch.cuda.synchronize()
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)


def test_release_reports_a_discarded_queued_update():
    """ADVICE r5 (api.hip ws_release): gm2_workspace_release with an output-layer Adam update still
    QUEUED (GM2_OPT_DEFER_OUTPUT_ADAM, no join) discards it and says so -- return 1 and a
    gm2_last_error message -- while a joined workspace releases with 0."""
    G, H, L, B = 1000, 128, 16, 256
    P, S = perturb_bn(*oracle_state(G, H, L, 75), seed=76)
    X = synth_x(B, G, 77)
    for join in (True, False):
        m = to_model(P, S, G, H, L, native.GM2_BF16)
        mat = ResidentMatrix(X)
        ws = m.workspace(native.GM2_BF16, B)
        ws.set_option(native.OPT_DEFER_OUTPUT_ADAM, 1)
        grads, mom, vel = torch.zeros_like(m.params), torch.zeros_like(m.params), torch.zeros_like(m.params)
        sc = scalars(beta=0.5, wgamma=0.0, lam=0.0, step=1)
        loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device="cuda")
        eps = torch.randn(B, L, generator=torch.Generator().manual_seed(78)).cuda()
        native.train_fwd_bwd(ws, native.make_batch(mat.data, mat.ld, None, B, eps), m.params, grads, m.bn, sc, loss)
        native.grad_norm(ws, m.params, grads, sc, loss)
        native.adam_step(ws, m.params, grads, mom, vel, sc)
        if join:
            ws.join()
        torch.cuda.synchronize()
        rc = native.lib().gm2_workspace_release(ws.ptr)
        if join:
            assert rc == 0
        else:
            assert rc == 1 and "discarded" in native.lib().gm2_last_error().decode()
        assert native.lib().gm2_workspace_release(ws.ptr) == 0  # (released: unknown state is a no-op)

