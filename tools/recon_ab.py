#!/usr/bin/env python3
"""A/B of libgm2 tuning options on the C2 step shape, interleaved rounds in one process; reports the
output-layer loss kernel's HIP-event time (KC_RECON_LOSS) and the step time.
Usage: python3 tools/recon_ab.py OPTION v1 v2 ...   (OPTION = recon_tile | small_split | gemm_pp | bn_epilogue | side_stream | small_waves)"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "genome-minimizer-2_amd"))
import bench  # noqa: E402
from gm2 import native  # noqa: E402
from gm2.data import ResidentMatrix, synthetic_pangenome  # noqa: E402
from gm2.model import VAE  # noqa: E402
from gm2.trainer import Adam  # noqa: E402

G, H, L, B = 55039, 1024, 64, 4096
dev = torch.device("cuda")
mat = ResidentMatrix(synthetic_pangenome(10000, G), device=dev)
torch.manual_seed(0)
model = VAE(G, H, L, device=dev, precision=native.GM2_BF16)
opt = Adam(model)
ws = model.workspace(native.GM2_BF16, B)
grads = torch.zeros_like(model.params)
scal = torch.tensor(bench.scalar_table(200), dtype=torch.float32, device=dev)
loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device=dev)
rows = torch.randperm(10000)[:B].to(torch.int32).to(dev)


def step(i):
    eps = torch.randn(B, L, device=dev)
    native.train_fwd_bwd(ws, native.make_batch(mat.data, mat.ld, rows, B, eps), model.params, grads, model.bn,
                         scal[i], loss)
    native.grad_norm(ws, model.params, grads, scal[i], loss)
    native.adam_step(ws, model.params, grads, opt.exp_avg, opt.exp_avg_sq, scal[i])


KEYS = {"recon_tile": native.OPT_RECON_TILE, "small_split": native.OPT_SMALL_SPLIT, "gemm_pp": native.OPT_GEMM_PP,
        "bn_epilogue": native.OPT_BN_EPILOGUE, "side_stream": native.OPT_SIDE_STREAM,
        "small_waves": native.OPT_SMALL_WAVES}


def main():
    opt_name = sys.argv[1] if len(sys.argv) > 1 else "recon_tile"
    vals = [int(v) for v in sys.argv[2:]] or [256, 128]
    key = KEYS[opt_name]
    res = {}
    for rnd in range(3):
        for tile in vals:
            native.set_option(key, tile)
            for i in range(2):
                step(i)
            torch.cuda.synchronize()
            native.timing_begin(native.KC_RECON_LOSS)
            t0 = time.perf_counter()
            for i in range(10):
                step(i + 2)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 10
            ms, n = native.timing_end()
            res.setdefault(tile, []).append((ms / n, dt * 1e3))
    for tile, v in res.items():
        k = sorted(x[0] for x in v)[len(v) // 2]
        st = sorted(x[1] for x in v)[len(v) // 2]
        print(f"{opt_name} {tile}: recon kernel {k * 1e3:.1f} us ({2 * B * H * G / (k * 1e-3) / 1e12:.0f} TF/s), step {st:.3f} ms")


if __name__ == "__main__":
    main()
