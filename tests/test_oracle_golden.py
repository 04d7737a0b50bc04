"""Pin the CPU oracle (oracle/vae_oracle.py) against the reference's own outputs.

The golden vectors were produced by tests/golden/make_golden.py importing /root/reference
(torch 2.10 CPU, 1 thread, MKL_CBWR=COMPATIBLE; the fixture meta records the CPU model and ISA).
The oracle restates the algorithm with the same fp32 ops in the same order, so at one thread, on
the same MKL code path (tests/conftest.py selects it) and on the fixture's CPU model it must match
BIT FOR BIT. On another CPU model torch's pointwise Adam update rounds ~0.3 % of parameters 1 ulp
differently (losses, gradients and Adam moments stay exact): golden_io.bit_pinned then switches
to the stated tolerances below, and the integer parts (RNG streams, epochs, counters) stay exact.
The explicit-gradient restatement (the math the HIP kernels implement) is checked against
autograd within fp32 rounding.
"""
import numpy as np
import pytest
import torch
from sklearn.model_selection import train_test_split

from golden_io import assert_pinned, bit_pinned, load, require_pinned
from oracle import vae_oracle as O


def _preset(name):
    return O.PRESETS[name]


def test_init_replays_reference_rng():
    g = load("init")
    for tag in ("a", "b"):
        G, H, L, seed = [int(v) for v in g[f"{tag}_dims"]]
        torch.manual_seed(seed)
        P = O.init_params(G, H, L)
        np.testing.assert_array_equal(O.flatten(P), g[f"{tag}_params"])
        np.testing.assert_array_equal(torch.rand(4).numpy(), g[f"{tag}_next"])


@pytest.mark.parametrize("preset", ["v0", "v1", "v2", "v3"])
def test_train_step_bit_exact(preset):
    g = load("steps")
    G, H, L, B, EPOCH, NEP = [int(v) for v in g["dims"]]
    torch.manual_seed(int(g[f"{preset}_init_seed"][0]))
    P = O.init_params(G, H, L)
    S = O.init_bn_state(H)
    ls = O.LossState(_preset(preset), NEP, counter=5)
    opt = O.AdamState(lr=1e-3)
    x = torch.tensor(g["X"], dtype=torch.float32)
    eps = torch.tensor(g[f"{preset}_eps"])
    parts, grads = O.train_step(P, S, ls, opt, x, eps, EPOCH)
    names = list(g[f"{preset}_loss_names"])
    got = np.array([parts[n] for n in names])
    assert_pinned(got.astype(np.float32), g[f"{preset}_losses"].astype(np.float32), g, "losses")
    assert_pinned(O.flatten(grads), g[f"{preset}_grads"], g, "grads")
    require_pinned(g)
    assert_pinned(O.flatten(P), g[f"{preset}_params"], g, "params")
    assert_pinned(O.flatten(opt.m), g[f"{preset}_exp_avg"], g, "exp_avg")
    assert_pinned(O.flatten(opt.v), g[f"{preset}_exp_avg_sq"], g, "exp_avg_sq")
    bn = np.concatenate([S[k].reshape(-1).numpy() for k in g["bn_keys"]])
    assert_pinned(bn, g[f"{preset}_bn"], g, "bn")


def _prebn_bias_mask(G, H, L):
    """Linear biases feeding a BatchNorm: their exact gradient is 0, the computed one is pure
    rounding noise (SURVEY.md §7 'Hard parts'), so they are compared with an absolute bound."""
    m = []
    for n, shp in O.param_specs(G, H, L):
        k = int(np.prod(shp))
        prebn = n.endswith(".bias") and n.split(".")[0] in ("encoder", "decoder") and \
            n.split(".")[1] in ("0", "3", "6")
        m.append(np.full(k, prebn))
    return np.concatenate(m)


@pytest.mark.parametrize("preset", ["v0", "v1", "v2", "v3"])
def test_manual_gradients_match_autograd(preset):
    g = load("steps")
    G, H, L, B, EPOCH, NEP = [int(v) for v in g["dims"]]
    torch.manual_seed(int(g[f"{preset}_init_seed"][0]))
    P = O.init_params(G, H, L)
    S = O.init_bn_state(H)
    pr = _preset(preset)
    ls = O.LossState(pr, NEP, counter=5)
    beta = ls.beta(EPOCH)
    wg = pr.weight * ls.gamma(EPOCH) if pr.gamma_start is not None else 0.0
    lam = pr.lambda_l1 or 0.0
    x = torch.tensor(g["X"], dtype=torch.float32)
    eps = torch.tensor(g[f"{preset}_eps"])
    G_ = O.flatten(O.manual_grads(P, S, x, eps, beta, wg, lam))
    ref = g[f"{preset}_raw_grads"]
    mask = _prebn_bias_mask(G, H, L)
    scale = np.abs(ref[~mask]).max()
    assert np.abs(G_[~mask] - ref[~mask]).max() <= 2e-5 * scale
    assert np.abs(G_[mask]).max() <= 1e-4 * scale and np.abs(ref[mask]).max() <= 1e-4 * scale


@pytest.mark.parametrize("preset", ["v0", "v1", "v2", "v3"])
def test_preset_trainer_bit_exact(preset):
    g = load("trainer")
    require_pinned(g)
    G, H, L, N, BS, NEP = [int(v) for v in g["dims"]]
    data = torch.tensor(g["data"], dtype=torch.float32)
    torch.manual_seed(int(g[f"{preset}_seed"][0]))
    P = O.init_params(G, H, L)
    S = O.init_bn_state(H)
    tr, va, ep = O.run_preset(P, S, _preset(preset), NEP, data[g["train_idx"]], data[g["val_idx"]], BS)
    assert ep == int(g[f"{preset}_epochs"][0])
    if bit_pinned(g):
        np.testing.assert_array_equal(np.array(tr), g[f"{preset}_train_losses"])
        np.testing.assert_array_equal(np.array(va), g[f"{preset}_val_losses"])
        np.testing.assert_array_equal(O.flatten(P), g[f"{preset}_params"])
    else:
        # Off the fixture's host the 1-ulp differences of the Adam update (golden_io.bit_pinned)
        # compound over the epochs. Stated trajectory bars: per-epoch losses within 1e-4 relative
        # (observed 1.4e-5 on an Intel Xeon); parameters: the median within 1e-6 and the 99th
        # percentile within 5e-4 (observed 1e-7 / 1.3e-4), and every one within 2 x steps x lr --
        # weights of all-zero input columns and biases feeding a BatchNorm have pure-noise
        # gradients that Adam turns into O(lr) steps of either sign.
        np.testing.assert_allclose(np.array(tr), g[f"{preset}_train_losses"], rtol=1e-4)
        np.testing.assert_allclose(np.array(va), g[f"{preset}_val_losses"], rtol=1e-4)
        d = np.abs(O.flatten(P) - g[f"{preset}_params"])
        steps = NEP * -(-len(g["train_idx"]) // BS)
        assert np.median(d) <= 1e-6 and np.quantile(d, 0.99) <= 5e-4
        assert d.max() <= 2 * steps * 1e-3
    # the RNG stream position is exact integer state: bit-exact on every host
    np.testing.assert_array_equal(torch.rand(3).numpy(), g[f"{preset}_rng_after"])
    assert all(int(S[b + ".num_batches_tracked"]) == n for b, n in zip(O.BNS, g[f"{preset}_nbt"]))


def _sampling_state(g, tag, G, H, L):
    P = O.init_params(G, H, L)  # encoder part irrelevant for decode
    S = O.init_bn_state(H)
    for k in g.files:
        if k.startswith(tag + "_sd/"):
            name = k[len(tag) + 4:]
            t = torch.tensor(g[k])
            (P if name in P else S)[name] = t
    return P, S


@pytest.mark.parametrize("tag", ["s", "p"])
def test_sampling_bit_exact(tag):
    g = load("sampling")
    G, H, L, N = [int(v) for v in g[f"{tag}_dims"]]
    P, S = _sampling_state(g, tag, G, H, L)
    p = O.sample_decode(P, S, torch.tensor(g[f"{tag}_z"])).numpy()
    assert_pinned(p, g[f"{tag}_p"], g, "p")
    # the fixtures are band-free (make_golden.py chooses them so), so the masks are exact everywhere
    np.testing.assert_array_equal((p > 0.5).astype(np.uint8), g[f"{tag}_mask"])
    # fp64 logit restatement and the logit-threshold form of the mask
    l64 = O.decode_logits64(P, S, torch.tensor(g[f"{tag}_z"])).numpy()
    np.testing.assert_allclose(l64, g[f"{tag}_logit64"], rtol=0, atol=1e-9)
    fm = g[f"{tag}_focused_mask"]
    pf = O.sample_decode(P, S, torch.tensor(g[f"{tag}_focused_z"])).numpy()
    np.testing.assert_array_equal((pf > 0.5).astype(np.uint8), fm)


def test_threshold_constant():
    g = load("numerics")
    x = g["thr_x"]
    np.testing.assert_array_equal((x > O.MASK_LOGIT_THRESHOLD).astype(np.uint8), g["thr_mask"])


@pytest.mark.parametrize("tgt", [0, 1])
def test_bce_semantics(tgt):
    g = load("numerics")
    l = torch.tensor(g["bce_logits"], requires_grad=True)
    p = torch.sigmoid(l)
    x = torch.full_like(p, float(tgt))
    loss = torch.nn.functional.binary_cross_entropy(p, x, reduction="sum")
    loss.backward()
    np.testing.assert_array_equal(l.grad.numpy(), g[f"bce_grad_t{tgt}"])
    # explicit element formula (what the fused epilogue computes)
    pn = torch.sigmoid(torch.tensor(g["bce_logits"]))
    if tgt:
        e = -torch.clamp(torch.log(pn), min=-100)
    else:
        e = -torch.clamp(torch.log1p(-pn), min=-100)
    # the reference's log/log1p come from vectorised (Sleef) or scalar libm paths depending on
    # tensor length, so elements agree to 1 ulp, not bitwise, even within torch itself
    np.testing.assert_allclose(e.numpy(), g[f"bce_elem_t{tgt}"], rtol=5e-7, atol=0)
    dp = (pn - tgt) / torch.clamp((1 - pn) * pn, min=1e-12)
    np.testing.assert_array_equal((dp * (1 - pn) * pn).numpy(), g[f"bce_grad_t{tgt}"])


def test_schedules():
    g = load("numerics")
    rows = []
    for (st, lo, hi, Tp, nep) in [("linear", 0.1, 1.0, 10, 7), ("cosine", 0.0, 1.0, 10, 7),
                                  ("cosine", 0.1, 1.0, 50, 7), ("constant", 0.1, 0.7, 10, 7)]:
        ls = O.LossState(O.Preset("x", st, lo, hi, T=Tp), nep)
        for epoch in range(4):
            for _ in range(3):
                rows.append(ls.beta(epoch))
    np.testing.assert_allclose(np.array(rows), g["sched_beta"], rtol=1e-15, atol=0)
    ls = O.LossState(O.Preset("x", "linear", 0, 1, gamma_start=2.0, gamma_end=0.1, weight=1.5), 9)
    gam = [ls.preset.weight * ls.gamma(e) for e in range(12)]
    np.testing.assert_allclose(np.array(gam), g["sched_gamma"], rtol=1e-15, atol=0)


def test_split_sizes():
    g = load("numerics")
    for n, a, b, c, s1, s2, s3 in g["split_sizes"]:
        tr, tmp = train_test_split(np.arange(n), test_size=0.3, random_state=12345)
        va, te = train_test_split(tmp, test_size=0.3333, random_state=12345)
        assert (len(tr), len(va), len(te)) == (a, b, c)
        assert (tr[:5].sum(), va[:5].sum(), te[:5].sum()) == (s1, s2, s3)
