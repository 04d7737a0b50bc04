"""Shared helpers for the @pytest.mark.gpu parity tests (HIP path vs the CPU oracle)."""
import numpy as np
import torch

from gm2 import native
from gm2.model import VAE
from oracle import vae_oracle as O


def oracle_state(G, H, L, seed):
    torch.manual_seed(seed)
    P = O.init_params(G, H, L)
    S = O.init_bn_state(H)
    return P, S


def perturb_bn(P, S, seed):
    """Non-trivial BN affine params / running stats (fresh init has gamma=1, beta=0, rm=0, rv=1)."""
    g = torch.Generator().manual_seed(seed)
    for bn in O.BNS:
        H = P[bn + ".weight"].shape[0]
        P[bn + ".weight"] = 0.8 + 0.4 * torch.rand(H, generator=g)
        P[bn + ".bias"] = 0.2 * torch.rand(H, generator=g) - 0.1
        S[bn + ".running_mean"] = 0.4 * torch.rand(H, generator=g) - 0.2
        S[bn + ".running_var"] = 0.5 + torch.rand(H, generator=g)
    return P, S


def to_model(P, S, G, H, L, prec):
    m = VAE(G, H, L, precision=prec, init=False)
    sd = {}
    for k, v in P.items():
        sd[k] = v
    for k, v in S.items():
        sd[k] = v
    m.load_state_dict(sd)
    return m


def synth_x(n, g, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    f = rng.beta(0.1, 1.0, size=g)
    f[rng.random(g) < 0.15] = 0.98
    return (rng.random((n, g)) < f[None, :]).astype(np.uint8)


def flat(d, names):
    return torch.cat([d[n].detach().reshape(-1).float().cpu() for n in names])


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def scalars(beta=0.5, wgamma=0.0, lam=0.0, lr=1e-3, step=1, max_norm=1.0, b1=0.9, b2=0.999, eps=1e-8):
    v = np.zeros(native.NUM_SCALARS)
    v[native.S_BETA], v[native.S_WGAMMA], v[native.S_LAMBDA] = beta, wgamma, lam
    v[native.S_NEG_STEP] = -(lr / (1 - b1 ** step))
    v[native.S_BC2_SQRT] = np.sqrt(1 - b2 ** step)
    v[native.S_MAX_NORM] = max_norm
    v[native.S_ONE_MINUS_B1], v[native.S_BETA2], v[native.S_ONE_MINUS_B2], v[native.S_ADAM_EPS] = 1 - b1, b2, 1 - b2, eps
    return torch.tensor(v, dtype=torch.float32).cuda()
