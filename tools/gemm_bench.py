#!/usr/bin/env python3
"""GEMM microbenchmark: the v0 training step's GEMM shapes (B=4096, G=55,039, H=1024, L=64) through
gm2_gemm with the hot path's own plan, timed per kernel with HIP events (KC_GEMM_STORE), both GEMM
main loops (GM2_OPT_GEMM_PP 0/1) interleaved in one process (methodology rule: A/B in one process).
Usage: python3 tools/gemm_bench.py [reps] [rounds]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "genome-minimizer-2_amd"))
from gm2 import native  # noqa: E402

B, G, H, L = 4096, 55040, 1024, 64
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda")
bf = torch.bfloat16
# (name, pk, qk, M, N, K): P(m,k) from P [M][K] if pk else [K][M]; Q likewise
shapes = [
    ("enc0 fwd  X.W0^T", 1, 1, B, H, G),
    ("dA5  dL.W9     ", 1, 0, B, H, G),
    ("dW9  dL^T.A5   ", 0, 0, G, H, B),
    ("dWe0 dY^T.X    ", 0, 0, H, G, B),
    ("dWe0 dYT.X  nn ", 1, 0, H, G, B),
    ("hid fwd A.W^T  ", 1, 1, B, H, H),
    ("hid dX dY.W    ", 1, 0, B, H, H),
    ("hid dW dY^T.A  ", 0, 0, H, H, B),
]
for name, pk, qk, M, N, K in shapes:
    Mp, Np = -(-M // 128) * 128, -(-N // 128) * 128
    P = (torch.rand((Mp, K) if pk else (K, Mp), device=dev) * 2 - 1).to(bf)
    Q = (torch.rand((Np, K) if qk else (K, Np), device=dev) * 2 - 1).to(bf)
    Cout = torch.empty(M, N, device=dev)
    ldp = K if pk else Mp
    ldq = K if qk else Np
    slab = torch.empty(8 * M * N + 4, device=dev)
    res = {0: [], 1: []}
    for r in range(rounds):
        for pp in (0, 1):
            native.set_option(native.OPT_GEMM_PP, pp)
            for _ in range(2):
                native.gemm(native.GM2_BF16, P, ldp, Q, ldq, Cout, N, M, N, K, -1, slab, pk, qk)
            torch.cuda.synchronize()
            native.timing_begin(native.KC_GEMM_STORE)
            for _ in range(reps):
                native.gemm(native.GM2_BF16, P, ldp, Q, ldq, Cout, N, M, N, K, -1, slab, pk, qk)
            ms, n = native.timing_end()
            res[pp].append(ms / n)
    line = f"{name} M={M:6d} N={N:6d} K={K:6d}"
    for pp in (0, 1):
        t = sorted(res[pp])[len(res[pp]) // 2]
        tf = 2.0 * M * N * K / (t * 1e-3) / 1e12
        line += f" | pp={pp} {t*1e3:8.1f} us {tf:7.1f} TF/s"
    print(line, flush=True)
    del P, Q, Cout, slab
native.set_option(native.OPT_GEMM_PP, 0)
