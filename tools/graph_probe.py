#!/usr/bin/env python3
"""Probe: the v0 training step replayed from HIP graphs (one captured graph per step: each step's
rows / eps / scalar row / loss slot are its own buffers, so no per-step copies) against the same
steps launched eagerly, on the bench's workload (resident synthetic 10,000 x 55,039 matrix).
Both runs start from the same init; their loss records must be identical.
Usage: python3 tools/graph_probe.py [batch] [steps] [warmup]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "genome-minimizer-2_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gm2 import native  # noqa: E402
from gm2.data import ResidentMatrix, synthetic_pangenome  # noqa: E402
from gm2.model import VAE  # noqa: E402
from gm2.trainer import Adam  # noqa: E402
from bench import scalar_table  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
W = int(sys.argv[3]) if len(sys.argv) > 3 else 3
G, H, L, S = 55039, 1024, 64, 10000
dev = torch.device("cuda")
x = synthetic_pangenome(S, G, seed=12345)
mat = ResidentMatrix(x, device=dev)
res = mat.operands(native.GM2_BF16)


def run(graph):
    torch.manual_seed(0)
    model = VAE(G, H, L, device=dev, precision=native.GM2_BF16)
    opt = Adam(model, lr=1e-3)
    ws = model.workspace(native.GM2_BF16, B)
    grads = torch.zeros_like(model.params)
    n = W + K
    tab = scalar_table(n, "v0")
    tab[:, native.S_NORM_AHEAD] = 1.0
    scal = torch.tensor(tab, dtype=torch.float32, device=dev)
    g = torch.Generator().manual_seed(100)
    rows = torch.cat([torch.randperm(S, generator=g)[:B] for _ in range(n)]).to(torch.int32).to(dev)
    torch.manual_seed(1)
    eps = torch.randn(n, B, L, device=dev)
    loss = torch.zeros(n, native.LOSS_SLOTS, dtype=torch.float64, device=dev)
    ws.set_option(native.OPT_DEFER_OUTPUT_ADAM, 1)
    ws.set_option(native.OPT_GRAD_BUCKETS, 0)
    batches = [native.make_batch(mat.data, mat.ld, rows[i * B:(i + 1) * B], B, eps[i], resident=res) for i in range(n)]

    def step(i):
        native.train_fwd_bwd(ws, batches[i], model.params, grads, model.bn, scal[i], loss[i])
        native.grad_norm(ws, model.params, grads, scal[i], loss[i])
        native.adam_step(ws, model.params, grads, opt.exp_avg, opt.exp_avg_sq, scal[i])

    for i in range(W):
        step(i)
    ws.join()
    torch.cuda.synchronize()
    graphs = []
    if graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        t = time.perf_counter()
        for i in range(W, n):
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                step(i)
            graphs.append(gr)
        print(f"captured {len(graphs)} graphs in {time.perf_counter() - t:.2f} s", flush=True)
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    if graph:
        for gr in graphs:
            gr.replay()
    else:
        for i in range(W, n):
            step(i)
    ws.join()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    out = loss.cpu().numpy().copy()
    p = model.params.float().sum().item()
    del graphs, model, opt, ws, grads
    torch.cuda.empty_cache()
    return el / K * 1e3, out, p


for rep in range(2):
    me, le, pe = run(False)
    mg, lg, pg = run(True)
    same = np.array_equal(le, lg)
    print(f"B={B} eager {me:.3f} ms/step  graph {mg:.3f} ms/step  losses identical {same}  "
          f"param sums {pe!r} {pg!r}", flush=True)
    if not same:
        d = np.abs(le - lg)
        print("max loss diff per slot", d.max(axis=0)[:5], "first differing step", int(np.argmax(d.max(axis=1) > 0)))
