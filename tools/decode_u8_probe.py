#!/usr/bin/env python3
"""Probe: the sampling decode's two output forms on the bench's trained v1 checkpoint (C3 dims) --
gm2_decode_mask (u8 masks, what extras.sample_from_model returns) vs gm2_decode_bits (packed bits,
what main.py and the bench use) -- per 65,536-genome chunk, timed with HIP events, and the masks
compared (the u8 mask must equal the unpacked bits).  Usage: python3 tools/decode_u8_probe.py [reps]"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "genome-minimizer-2_amd"))
sys.path.insert(0, os.path.join(HERE, ".."))
import bench  # noqa: E402
from gm2 import native  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
sys.argv = [sys.argv[0]]
a = bench.parse()
dev = torch.device("cuda")
G, H, L, n = a.genes, 512, 32, 65536
m = bench.train_v1_checkpoint(a, dev, G, H, L)
m.eval()
ws = m.workspace(native.GM2_F32, n)
ldb = native.packed_row_bytes(G)
bits = torch.empty(n, ldb, dtype=torch.uint8, device=dev)
mask = torch.empty(n, G, dtype=torch.uint8, device=dev)
torch.manual_seed(0)
z = torch.randn(n, L, device=dev)


def timed(f):
    f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


tb = timed(lambda: native.decode_bits(ws, m.params, m.bn, z, n, bits, ldb))
tm = timed(lambda: native.decode_mask(ws, m.params, m.bn, z, n, mask, G))
unpacked = np.unpackbits(bits.cpu().numpy(), axis=1, count=G, bitorder="little")
same = np.array_equal(unpacked, mask.cpu().numpy())
print(f"decode of {n} genomes (G={G}, H={H}): bits {tb:.3f} ms, u8 {tm:.3f} ms; masks equal: {same}", flush=True)
sys.exit(0 if same else 1)
