#!/usr/bin/env python3
"""Generate tests/golden/sampling_split.npz by IMPORTING the reference (run here only: /root/reference
does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_sampling_split.py

A reference-produced sampling fixture at a shape and scale where the gated decode's bf16x3 output
layer (api.hip decode_split3, GM2_OPT_SAMPLE_SPLIT) runs on most tiles: G = 3,000 genes, hidden 512,
latent 32, N = 1,024 genomes (4 x 12 tiles of 256 x 256). The masks are `sample_from_model`'s three
lines (extras.py:196-201: z = randn(N, L); p = model.decode(z); p > 0.5) against the reference's own
`VAE.decode` (model.py:106-107) on CPU in eval mode after load_state_dict, as make_golden.py's
sampling fixture. Scale choices (decoder-only state, random init of the reference module):
  * decoder.7 BatchNorm gamma in [0.4, 0.6] keeps the last activations' norms ~7, so the split
    bound 4.62e-5 x max||a_r|| x max||w_g|| stays well under the gate (1e-3) on most tiles;
  * gene block 3 (genes 768..1023) has its output weights x 25 and genome block 2 (rows
    512..767) its z x 20: the tiles of that row or column fail the bound, so the gated decode runs
    a mix of split and exact tiles (the fixture records the per-tile verdict computed from the
    reference module's fp64 activations, with the margin to the bound).
  * size: the decoder's weights and z are rounded to fp16-representable values BEFORE the reference
    decodes (so they are stored losslessly as fp16; they keep 11 significant bits, so the split's
    lo parts are non-zero), the masks are stored packed (numpy packbits, little bit order), and
    the fp64 logits (a double copy of the module) only where |logit| <= 2e-3 (flat index, value):
    every other logit is farther from the threshold.
"""
import json
import math
import os
import sys

import numpy as np

REF = "/root/reference"
OUT = os.environ.get("GM2_GOLDEN_OUT") or os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
os.environ["MKL_CBWR"] = "COMPATIBLE"

import torch  # noqa: E402

torch.set_num_threads(1)

from src.genome_minimizer_2.training.model import VAE  # noqa: E402

SPLIT_UNIT, SPLIT_BOUND = 4.62e-5, 1e-3  # gm2_kernels.hpp kSplitUnit / kSplitBound


def main():
    G, H, L, N = 3000, 512, 32, 1024
    torch.manual_seed(31)
    model = VAE(G, H, L)
    with torch.no_grad():
        for mod in model.decoder:
            if isinstance(mod, torch.nn.BatchNorm1d):
                mod.running_mean.uniform_(-0.2, 0.2)
                mod.running_var.uniform_(0.5, 1.5)
                mod.weight.uniform_(0.8, 1.2)
                mod.bias.uniform_(-0.1, 0.1)
        model.decoder[7].weight.uniform_(0.4, 0.6)
        model.decoder[9].weight[768:1024] *= 25.0
        model.decoder[9].bias.uniform_(-0.3, 0.3)
        for k, v in model.state_dict().items():
            if k.startswith("decoder.") and v.is_floating_point():
                v.copy_(v.half().float())
    model.eval()
    torch.manual_seed(1031)
    with torch.no_grad():
        z = torch.randn(N, L)
        z[512:768] *= 20.0
        z = z.half().float()
        p = model.decode(z).numpy()  # the reference's fp32 decode (extras.py:198)
    mask = (p > 0.5).astype(np.uint8)  # extras.py:200-201
    with torch.no_grad():
        md = VAE(G, H, L).double()
        md.load_state_dict({k: (v.double() if v.is_floating_point() else v) for k, v in model.state_dict().items()})
        md.eval()
        a64 = md.decoder[:9](z.double())
        logit64 = md.decoder[9](a64).numpy()
        w64 = md.decoder[9].weight.numpy()
    an = np.linalg.norm(a64.numpy(), axis=1)
    wn = np.linalg.norm(w64, axis=1)
    rb, gb = (N + 255) // 256, (G + 255) // 256
    amax = np.array([an[i * 256:(i + 1) * 256].max() for i in range(rb)])
    wmax = np.array([wn[j * 256:(j + 1) * 256].max() for j in range(gb)])
    bound = SPLIT_UNIT * 1.01 * amax[:, None] * wmax[None, :]
    verdict = bound <= SPLIT_BOUND
    margin = np.abs(np.log(bound / SPLIT_BOUND)).min()
    print(np.array2string(bound, precision=2, max_line_width=200))
    assert margin > 0.15, f"a tile's bound is within {margin:.3f} (log) of the gate: rescale"
    assert verdict.sum() > 0 and (~verdict).sum() > 0
    print(f"split tiles {int(verdict.sum())} / {verdict.size}; bound range {bound.min():.3g} .. {bound.max():.3g}; "
          f"log margin {margin:.3f}; |logit64| <= 1e-3: {int((np.abs(logit64) <= 1e-3).sum())}")
    near = np.flatnonzero(np.abs(logit64) <= 2e-3)
    out = {"dims": np.array([G, H, L, N]), "z16": z.numpy().astype(np.float16),
           "mask_bits": np.packbits(mask, axis=1, bitorder="little"), "near_idx": near.astype(np.int32),
           "near_logit64": logit64.reshape(-1)[near], "split_verdict": verdict.astype(np.uint8), "split_bound": bound}
    for k, v in model.state_dict().items():
        if k.startswith("decoder."):
            a = v.numpy()
            if v.is_floating_point():
                assert np.array_equal(a.astype(np.float16).astype(np.float32), a)
                a = a.astype(np.float16)
            out["sd/" + k] = a
    meta = {"torch": torch.__version__, "threads": 1, "generator": "tests/golden/make_golden_sampling_split.py",
            "mkl_cbwr": os.environ["MKL_CBWR"], "split_unit": SPLIT_UNIT, "split_bound": SPLIT_BOUND}
    np.savez_compressed(os.path.join(OUT, "sampling_split.npz"), meta=json.dumps(meta), **out)
    print("sampling_split.npz", os.path.getsize(os.path.join(OUT, "sampling_split.npz")))


if __name__ == "__main__":
    main()
