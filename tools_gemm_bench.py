#!/usr/bin/env python3
"""GEMM microbenchmark: the v0 training step's GEMM shapes (B=4096, G=55,039, H=1024, L=64) through
gm2_gemm with the hot path's own plan, timed per kernel with HIP events (KC_GEMM_STORE).
Usage: python3 tools_gemm_bench.py [reps]"""
import sys
import torch
sys.path.insert(0, "genome-minimizer-2_amd")
from gm2 import native

B, G, H, L = 4096, 55040, 1024, 64
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda")
bf = torch.bfloat16
# (name, pk, qk, M, N, K): P(m,k) from P [M][K] if pk else [K][M]; Q likewise
shapes = [
    ("enc0 fwd  X.W0^T", 1, 1, B, H, G),
    ("dA5  dL.W9     ", 1, 0, B, H, G),
    ("dW9  dL^T.A5   ", 0, 0, G, H, B),
    ("dWe0 dY^T.X    ", 0, 0, H, G, B),
    ("hid fwd A.W^T  ", 1, 1, B, H, H),
    ("hid dX dY.W    ", 1, 0, B, H, H),
    ("hid dW dY^T.A  ", 0, 0, H, H, B),
]
for name, pk, qk, M, N, K in shapes:
    Mp, Np = -(-M // 128) * 128, -(-N // 128) * 128
    P = (torch.randn(Mp, K, device=dev) if pk else torch.randn(K, Mp, device=dev)).to(bf)
    Q = (torch.randn(Np, K, device=dev) if qk else torch.randn(K, Np, device=dev)).to(bf)
    Cout = torch.empty(M, N, device=dev)
    ldp = K if pk else Mp
    ldq = K if qk else Np
    # split plans only arise for shapes with < 256 big tiles: 8 slices of M x N is the bound
    slab = torch.empty(8 * M * N, device=dev) if M * N <= 8 * B * H else None
    for _ in range(2):
        native.gemm(native.GM2_BF16, P, ldp, Q, ldq, Cout, N, M, N, K, -1, slab, pk, qk)
    torch.cuda.synchronize()
    native.timing_begin(native.KC_GEMM_STORE)
    for _ in range(reps):
        native.gemm(native.GM2_BF16, P, ldp, Q, ldq, Cout, N, M, N, K, -1, slab, pk, qk)
    ms, n = native.timing_end()
    t = ms / n
    tf = 2.0 * M * N * K / (t * 1e-3) / 1e12
    # spot check vs torch (fp32 of the bf16 inputs) on a corner
    Pm = P[:256].float() if pk else P[:, :256].float().t()
    Qm = Q[:256].float() if qk else Q[:, :256].float().t()
    ref = Pm @ Qm.t()
    err = float((Cout[:256, :256] - ref).abs().max() / ref.abs().max())
    print(f"{name} M={M:6d} N={N:6d} K={K:6d}  {t*1e3:8.1f} us  {tf:7.1f} TF/s  err {err:.1e}", flush=True)
    del P, Q, Cout
