"""Run by tests/test_gpu_debug_build.py in a child process whose GM2_LIB_PATH selects the GM2_DEBUG
build (gm2/libgm2_debug.so): drives the kernels that follow index data and prints one JSON line with
the debug flag words read after each part (include/gm2_debug.h)."""
import ctypes as C
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "genome-minimizer-2_amd"), HERE):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gm2 import native  # noqa: E402
from gm2.data import ResidentMatrix  # noqa: E402
from gpu_helpers import oracle_state, scalars, synth_x, to_model  # noqa: E402


def flags():
    torch.cuda.synchronize()
    v = C.c_uint(0)
    native.check(native.lib().gm2_debug_flags(C.byref(v)), "gm2_debug_flags")
    return int(v.value)


def main():
    assert native.LIB_PATH.endswith("libgm2_debug.so"), native.LIB_PATH
    out = {"start": flags()}
    import __graft_entry__ as ge
    ge.smoke()  # f32 training step (gathered rows) + exact-fp32 decode, checked against the oracle
    out["smoke"] = flags()
    # bf16 training with zero-copy rows (the row tables of the input-layer GEMMs and the loss epilogue)
    G, H, L, B = 16384, 1024, 32, 1024
    S = 2 * B + 5
    P, Sb = oracle_state(G, H, L, 5)
    X = synth_x(S, G, 6)
    m = to_model(P, Sb, G, H, L, native.GM2_BF16)
    mat = ResidentMatrix(X)
    res = mat.operands(native.GM2_BF16)
    ws = m.workspace(native.GM2_BF16, B)
    grads = torch.zeros_like(m.params)
    gen = torch.Generator().manual_seed(7)
    rows = torch.randperm(S, generator=gen)[:B].to(torch.int32).cuda()
    eps = torch.randn(B, L, generator=gen).cuda()
    sc = scalars(beta=0.3)
    loss = torch.zeros(native.LOSS_SLOTS, dtype=torch.float64, device="cuda")
    native.train_fwd_bwd(ws, native.make_batch(mat.data, mat.ld, rows, B, eps, resident=res), m.params, grads, m.bn,
                         sc, loss)
    ws.join()
    out["zero_copy"] = flags()
    out["loss_finite"] = bool(torch.isfinite(loss[:3]).all().item())
    # a batch row index == S: the resident operands' zero row (memory-safe), but outside the matrix
    rows_bad = rows.clone()
    rows_bad[17] = S
    native.train_fwd_bwd(ws, native.make_batch(mat.data, mat.ld, rows_bad, B, eps, resident=res), m.params, grads,
                         m.bn, sc, loss)
    ws.join()
    out["bad_row"] = flags()
    # mask consumers: valid groups, then descending group offsets (the loop body never runs)
    n, Gm = 64, 1000
    ldb = native.packed_row_bytes(Gm) if hasattr(native, "packed_row_bytes") else ((Gm + 127) // 128) * 16
    bits = torch.randint(0, 256, (n, ldb), dtype=torch.uint8, device="cuda")
    goff = torch.tensor([0, 2, 5, 9], dtype=torch.int32, device="cuda")
    pos = torch.tensor([1, 7, 100, 200, 300, 5, 6, 7, 999], dtype=torch.int32, device="cuda")
    counts = torch.zeros(n, dtype=torch.int32, device="cuda")
    lib = native.lib()
    s = native.stream()
    native.check(lib.gm2_mask_count_groups(bits.data_ptr(), n, ldb, goff.data_ptr(), 3, pos.data_ptr(),
                                           counts.data_ptr(), s), "count_groups")
    offs = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    native.check(lib.gm2_mask_row_offsets(bits.data_ptr(), n, ldb, None, offs.data_ptr(), s), "row_offsets")
    idx = torch.zeros(int(offs[-1].item()) + 1, dtype=torch.int32, device="cuda")
    native.check(lib.gm2_mask_compact(bits.data_ptr(), n, ldb, None, offs.data_ptr(), idx.data_ptr(), s), "compact")
    out["masks"] = flags()
    goff_bad = torch.tensor([0, 5, 2, 9], dtype=torch.int32, device="cuda")
    native.check(lib.gm2_mask_count_groups(bits.data_ptr(), n, ldb, goff_bad.data_ptr(), 3, pos.data_ptr(),
                                           counts.data_ptr(), s), "count_groups")
    out["bad_groups"] = flags()
    print("DEBUGPROBE " + json.dumps(out))


if __name__ == "__main__":
    main()
