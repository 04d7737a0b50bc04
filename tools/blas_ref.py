#!/usr/bin/env python3
"""Calibration only (not product code): hipBLASLt (torch.matmul, bf16 in, fp32 accumulate) on the
hot path's GEMM shapes, to set what a vendor library reaches next to libgm2's GEMMs
(tools/gemm_bench.py prints the same shapes for libgm2)."""
import torch

SHAPES = [  # name, M, N, K, layout of (P, Q): "nt" = both K-contiguous, "nn"/"tn" otherwise
    ("enc0 fwd  X.W0^T", 4096, 1024, 55040),
    ("dA5  dL.W9     ", 4096, 1024, 55040),
    ("dW9  dL^T.A5   ", 55040, 1024, 4096),
    ("dWe0 dY^T.X    ", 1024, 55040, 4096),
    ("recon A5.W9^T  ", 55040, 4096, 1024),
    ("hid  A.W^T     ", 4096, 1024, 1024),
]


def bench(f, it=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def main():
    dev = "cuda"
    for name, M, N, K in SHAPES:
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        b = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        at = a.t().contiguous().t()  # same values, MN-major storage
        for lay, (x, y) in (("nt", (a, b.t())), ("tn", (at, b.t()))):
            us = bench(lambda: torch.matmul(x, y))
            print(f"{name} M={M:6d} N={N:6d} K={K:6d} {lay}: {us:8.1f} us {2 * M * N * K / us / 1e6:8.1f} TF/s",
                  flush=True)
        del a, b, at
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
