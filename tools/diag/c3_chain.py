"""Diagnostic (GPU): where does libgm2's exact-fp32 C3 step lose accuracy against torch fp32?
Runs the oracle's explicit backward (manual_grads_emulated's math) three ways on the C3 shapes
(v1: G = 55,039, H = 512, L = 32, w*gamma = 1, B = 4096): fp64 (exact), fp32 with torch matmuls,
fp32 with every matmul done by libgm2's f32 GEMM (gm2_gemm, hot-path plan); and the libgm2 step
itself. Prints the per-tensor fro errors of each against exact."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "genome-minimizer-2_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
from gm2 import native  # noqa: E402
from gm2.data import ResidentMatrix, synthetic_pangenome  # noqa: E402
from gpu_helpers import perturb_bn, scalars, to_model  # noqa: E402
from oracle import vae_oracle as O  # noqa: E402

G, H, L, B, WG, BETA = 55039, int(sys.argv[2]) if len(sys.argv) > 2 else 512, 32, 4096, \
    float(sys.argv[1]) if len(sys.argv) > 1 else 1.0, 0.1
dev = torch.device("cuda")
torch.manual_seed(2024)
P = O.init_params(G, H, L)
S = O.init_bn_state(H)
P, S = perturb_bn(P, S, 99)
Xh = synthetic_pangenome(B, G, seed=12345)
torch.manual_seed(5)
eps = torch.randn(B, L)


def gm2_mm(a, b):
    """a [M,K] @ b [K,N] in fp32 through gm2_gemm (P = a K-major, Q = b MN-major)."""
    M, K = a.shape
    N = b.shape[1]
    Kp = -(-K // 64) * 64
    Mp, Np = -(-M // 128) * 128, -(-N // 128) * 128
    A = torch.zeros(Mp, Kp, device=dev)
    A[:M, :K] = a
    Bm = torch.zeros(Kp, Np, device=dev)
    Bm[:K, :N] = b
    C = torch.empty(M, N, device=dev)
    slab = torch.empty(8 * M * N + 4, device=dev)
    native.gemm(native.GM2_F32, A, Kp, Bm, Np, C, N, M, N, Kp, -1, slab, True, False)
    return C


def chain(dt, mm, mm_long=None, on=None):
    mm_long = mm_long or mm
    BN_EPS = 1e-5
    on = on or dev
    Pd = {k: v.to(on, dt) for k, v in P.items()}
    x = torch.tensor(Xh, device=on, dtype=dt)
    e = eps.to(on, dt)
    cache = []
    Gr_fwd = {}

    def blk(lin, bn, a):
        f = mm_long if a.shape[1] > 4096 else mm
        y = f(a, Pd[lin + ".weight"].t().contiguous()) + Pd[lin + ".bias"]
        Gr_fwd["y." + lin] = y - y.mean(0)
        mean = y.mean(0)
        var = ((y - mean) ** 2).mean(0)
        invstd = 1.0 / torch.sqrt(var + BN_EPS)
        xhat = (y - mean) * invstd
        o = xhat * Pd[bn + ".weight"] + Pd[bn + ".bias"]
        cache.append((lin, bn, a, xhat, invstd, o))
        return torch.relu(o)
    h = x
    for i in range(3):
        h = blk(f"encoder.{3*i}", f"encoder.{3*i+1}", h)
    h2 = h
    mu = mm(h2, Pd["mean_layer.weight"].t().contiguous()) + Pd["mean_layer.bias"]
    lv = mm(h2, Pd["logvar_layer.weight"].t().contiguous()) + Pd["logvar_layer.bias"]
    std = torch.exp(0.5 * lv)
    z = mu + std * e
    h = z
    for i in range(3):
        h = blk(f"decoder.{3*i}", f"decoder.{3*i+1}", h)
    a5 = h
    logit = mm(a5, Pd["decoder.9.weight"].t().contiguous()) + Pd["decoder.9.bias"]
    p = torch.sigmoid(logit)
    Gr = {}
    dp = (p - x) / torch.clamp((1 - p) * p, min=1e-12) + WG
    dl = dp * (1 - p) * p
    Gr["decoder.9.weight"] = mm(dl.t().contiguous(), a5)
    da = mm_long(dl, Pd["decoder.9.weight"])
    Gr["dA5"] = da
    Gr.update(Gr_fwd)

    def blk_bwd(entry, da):
        lin, bn, a, xhat, invstd, o = entry
        do = da * (o > 0).to(dt)
        sdo = do.sum(0)
        sdx = (do * xhat).sum(0)
        Gr[bn + ".weight"] = sdx
        Gr[bn + ".bias"] = sdo
        dy = Pd[bn + ".weight"] * invstd / B * (B * do - sdo - xhat * sdx)
        Gr["dY." + lin] = dy
        Gr[lin + ".weight"] = mm(dy.t().contiguous(), a)
        return mm(dy, Pd[lin + ".weight"])
    for en in reversed(cache[3:]):
        da = blk_bwd(en, da)
    return Gr


ex = chain(torch.float64, lambda a, b: a @ b)
t32 = chain(torch.float32, lambda a, b: a @ b)
g32 = chain(torch.float32, gm2_mm)
gl = chain(torch.float32, lambda a, b: a @ b, gm2_mm)   # libgm2 only for the K = G GEMMs
torch.set_num_threads(16)
cpu = chain(torch.float32, lambda a, b: a @ b, on=torch.device("cpu"))  # the reference: torch CPU (MKL)
cpu = {k: v.to(dev) for k, v in cpu.items()}
gs = chain(torch.float32, gm2_mm, lambda a, b: a @ b)   # libgm2 only for the short-K GEMMs
m = to_model(P, S, G, H, L, native.GM2_F32)
mat = ResidentMatrix(Xh)
ws = m.workspace(native.GM2_F32, B)
grads = torch.zeros_like(m.params)
loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device=dev)
native.train_fwd_bwd(ws, native.make_batch(mat.data, mat.ld, None, B, eps.cuda()), m.params, grads, m.bn,
                     scalars(beta=BETA, wgamma=WG), loss)
torch.cuda.synchronize()
lib = {n: grads[m.offsets[i]:m.offsets[i + 1]].view(s) for i, (n, s) in enumerate(m.specs)}


def fro(a, b):
    return (a.double() - b.double()).norm().item() / max(b.double().norm().item(), 1e-300)


print(f"w*gamma = {WG}")
for k in ex:
    row = (f"{k:22s} torch32 {fro(t32[k], ex[k]):.3e}  gm2gemm32 {fro(g32[k], ex[k]):.3e}  "
           f"gm2 longK only {fro(gl[k], ex[k]):.3e}  gm2 shortK only {fro(gs[k], ex[k]):.3e}  "
           f"CPU-MKL32 {fro(cpu[k], ex[k]):.3e}")
    if k in lib:
        row += f"  libgm2 {fro(lib[k], ex[k]):.3e}"
    print(row)
