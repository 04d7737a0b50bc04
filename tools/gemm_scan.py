#!/usr/bin/env python3
"""Fixed vs per-K-step cost of the hidden-layer GEMM shape (M=4096, N=1024, nt, bf16): time
gm2_gemm over K = 64 .. 4096 (HIP events, KC_GEMM_STORE) and fit t = a + b * (K / 64)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "genome-minimizer-2_amd"))
from gm2 import native  # noqa: E402

dev = torch.device("cuda")
M, N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096, int(sys.argv[2]) if len(sys.argv) > 2 else 1024
Ks = [64, 128, 256, 512, 1024, 2048, 4096]
ts = []
for K in Ks:
    P = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    Q = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
    C = torch.empty(M, N, device=dev)
    for _ in range(3):
        native.gemm(native.GM2_BF16, P, K, Q, K, C, N, M, N, K, 1, None, 1, 1)
    torch.cuda.synchronize()
    res = []
    for r in range(3):
        native.timing_begin(native.KC_GEMM_STORE)
        for _ in range(20):
            native.gemm(native.GM2_BF16, P, K, Q, K, C, N, M, N, K, 1, None, 1, 1)
        ms, n = native.timing_end()
        res.append(ms / n * 1e3)
    t = sorted(res)[1]
    ts.append(t)
    print(f"M={M} N={N} K={K:5d}: {t:7.2f} us  {2 * M * N * K / (t * 1e-6) / 1e12:7.1f} TF/s", flush=True)
b, a = np.polyfit(np.array(Ks) / 64, np.array(ts), 1)
print(f"fit: {a:.2f} us fixed + {b:.3f} us per 64-deep K-step")
