#!/usr/bin/env python3
"""Benchmark: strain-vectors/sec of the v0 VAE training step on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], "C2"): v0 preset (hidden 1024, latent 64, linear KL anneal),
bf16 MFMA GEMMs with fp32 master weights, batch 4096 strain rows per GPU per step, synthetic
F4-shaped pan-genome matrix 10,000 strains x 55,039 genes resident in HBM (u8). One step = the
whole hot path of trainer.py:109-120 on one batch: row gather, encoder/decoder forward with
train-mode BatchNorm, reparameterisation, fused BCE/KL epilogues, full backward, gradient norm +
clip, Adam. N>1 (torchrun): one process per GPU, each rank steps its own 4096 rows, gradients
SUM-all-reduced over RCCL every step (weak scaling: value = all ranks' rows / max-rank time).
`python bench.py --gpus N` without a torchrun environment launches the N ranks itself (a child
`torch.distributed.run` process; this parent never touches the GPU) and exits with its code.

Also reported (extra fields, not `value`): sampling throughput of `--mode sample` for the v1 preset
(C3: 1e6 genomes from a v1 checkpoint trained on the synthetic matrix, decoded with the output layer
gated per 256 x 256 tile between one bf16 product over the rounded operands (the single tier), the
bf16x3 split and exact fp32, the certified band recomputed in fp64 (a list overflow recomputes its
blocks whole), thresholded into packed masks, essential genes counted on the device, masks + counts
copied to pinned host memory; the tier fractions and band counts are reported), the v1 / v2 / v3
training steps at C3 / C4's per-GPU dims (hidden 512, latent 32, gene abundance + L1, cosine KL for
v2 / v3), the C1 workload on the GPU (v0 at batch 64 and at the CLI default 32, F4 width), the same
training step in the other GEMM
precision (f32 next to the bf16 headline), the live-timed dominant kernel against the MFMA roofline,
and the CPU baseline (the oracle = the reference's algorithm on torch-CPU, fp32, all host threads,
the same v0 step at batch 4096 on the same matrix; plus the C1 batch-64 point), and the C5-shaped
step (configs[4]: v0 on the synthetic 100k-strain x 20k-gene matrix, 4096 rows per GPU, each rank
holding its 1/8 shard of 12,500 strains) with its own roofline entry. Every timed step must be
finite (losses and gradient norm): a non-finite step fails the run.
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "genome-minimizer-2_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, no sparsity)
PEAK_F32_TFLOPS = 157.3     # MI355X fp32 matrix peak
PEAK_HBM_GBS = 8000.0


def train_flops_per_vector(G, H, L):
    """2*(3*(2GH + 4H^2 + 3HL) - GH) (fwd + dX + dW; no dX for the input layer)."""
    return 2 * (3 * (2 * G * H + 4 * H * H + 3 * H * L) - G * H)


def decode_flops_per_genome(G, H, L):
    return 2 * (L * H + 2 * H * H + H * G)


DEFAULTS = dict(batch=4096, genes=55039, hidden=1024, latent=64, precision="bf16")


def pmc_traffic(a, kernel_prefix, grid=None, pattern="r*_pmc_traffic.json"):
    """HBM bytes per launch of `kernel_prefix` from the newest committed PMC summary matching
    `pattern` (profiles/rNN_pmc_traffic.json, written by tools/pmc.py from separate FETCH_SIZE /
    WRITE_SIZE rocprofv3 passes of this same command; the sample leg's kernels from
    rNN_pmc_sample_trained.json, the passes over the trained checkpoint it decodes from,
    tools/pmc_sample.sh). Only valid for the default workload; else None."""
    import glob
    if any(getattr(a, k) != v for k, v in DEFAULTS.items()):
        return None, None
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)))
    if not files:
        return None, None
    rows = [r for r in json.load(open(files[-1]))["kernels"] if r["kernel"].startswith(kernel_prefix)
            and (grid is None or r["grid"] == grid)]
    if not rows:
        return None, None
    return rows[0]["traffic_bytes"], os.path.relpath(files[-1], ROOT)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--genes", type=int, default=55039)
    ap.add_argument("--strains", type=int, default=10000)
    ap.add_argument("--hidden", type=int, default=1024)
    ap.add_argument("--latent", type=int, default=64)
    ap.add_argument("--precision", choices=["bf16", "f32"], default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sample", action="store_true")
    ap.add_argument("--sample-genomes", type=int, default=1000000)
    ap.add_argument("--copy-streams", type=int, default=1,
                    help="sample leg: copy streams the packed masks leave on (each a share of a chunk's rows)")
    ap.add_argument("--sample-train-epochs", type=int, default=10,
                    help="epochs of v1 training (lr 1e-3, batch 4096, the synthetic matrix) before the sample leg "
                         "decodes from that checkpoint; 0 = the untrained (xavier) model")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-f32-line", action="store_true")
    ap.add_argument("--no-prefetch", action="store_true",
                    help="N>1: gather each batch inside its own step (default: staged during the previous step)")
    ap.add_argument("--grad-exchange", choices=["f32", "bf16"], default="bf16",
                    help="N>1: dtype the big weight gradients are all-reduced in (gm2.ddp.GradSync)")
    ap.add_argument("--grid-cap", type=int, choices=range(8), default=None,
                    help="capped grid bits: output- (1) / input-layer (2) weight-gradient GEMMs, recon (4)")
    ap.add_argument("--input-chunks", type=int, choices=[1, 4], default=None,
                    help="input-layer weight-gradient launches (default: 4 under DDP, else 1)")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5-shaped (G=20,000) step line")
    ap.add_argument("--no-presets", action="store_true", help="skip the v1 / v2 / v3 step lines (C3 / C4 per GPU)")
    ap.add_argument("--no-adam-timing", action="store_true",
                    help="no live event pairs around the Adam launches (roofline_hbm then null)")
    ap.add_argument("--no-c1", action="store_true", help="skip the batch-64 / batch-32 GPU lines (C1 workload)")
    ap.add_argument("--defer-adam", type=int, default=None,
                    help="output layer's Adam update launched beside the next step's hidden layers on this many "
                         "workgroups per CU, 0 = not deferred (GM2_OPT_DEFER_OUTPUT_ADAM; bit-identical; default 1, as the "
                         "trainer: 3.34 -> 3.25 ms/step on one GPU, profiles/r03_schedule_ab.txt)")
    ap.add_argument("--host-timing", action="store_true",
                    help="print the host's enqueue time per timed step to stderr (diagnostic)")
    ap.add_argument("--no-zero-copy", action="store_true",
                    help="gather each step's rows instead of reading the resident operands in place")
    ap.add_argument("--grad-buckets", type=int, choices=[0, 1], default=0,
                    help="record gradient-bucket events on one GPU too (GM2_OPT_GRAD_BUCKETS; always 1 under DDP)")
    ap.add_argument("--recon-tile", type=int, choices=[0, 128, 256], default=None,
                    help="tile of the output-layer loss GEMM: 0 plan, 128 / 256 force (GM2_OPT_RECON_TILE)")
    ap.add_argument("--c5-strains", type=int, default=12500,
                    help="strains resident per rank for the C5 line (the 1/8 shard of 100,000)")
    return ap.parse_args()


def launch_ranks(a):
    """`--gpus N` outside torchrun: start N ranks through a child torch.distributed.run (one process
    per GPU, 127.0.0.1 rendezvous) and return its exit code. Nothing here initialises the GPU
    (torch.cuda.device_count does not), so the parent never holds a device context."""
    backend = os.environ.get("GM2_DIST_BACKEND", "nccl")
    if backend == "nccl" and torch.cuda.device_count() < a.gpus:
        print(f"bench.py: --gpus {a.gpus} but {torch.cuda.device_count()} GPU(s) visible "
              "(GM2_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs)", file=sys.stderr)
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def cpu_baseline(x_u8, G, H, L, budget_s, batch):
    """The oracle (reference algorithm: torch-CPU fp32 autograd, the reference's op order) on the
    box's host cores, SAME workload as the GPU line: v0 preset, batch `batch` rows of the same
    synthetic pan-genome matrix, fwd + bwd + clip + Adam per step; warm-up step, then as many
    timed steps as fit `budget_s` (at least one)."""
    sys.path.insert(0, ROOT)
    from oracle import vae_oracle as O
    threads = torch.get_num_threads()
    torch.manual_seed(0)
    P = O.init_params(G, H, L)
    S = O.init_bn_state(H)
    g = torch.Generator().manual_seed(7)
    n_rows = x_u8.shape[0]

    def xb():
        idx = torch.randperm(n_rows, generator=g)[:batch].numpy()
        return torch.from_numpy(x_u8[idx].astype(np.float32))
    ls = O.LossState(O.PRESETS["v0"], 10000)
    opt = O.AdamState()
    x = xb()
    t0 = time.perf_counter()
    O.train_step(P, S, ls, opt, x, torch.randn(batch, L), 0)  # warm-up
    first = time.perf_counter() - t0
    n = max(1, min(50, int(budget_s / max(first, 1e-3))))
    xs = [xb() for _ in range(n)]
    t0 = time.perf_counter()
    for i in range(n):
        O.train_step(P, S, ls, opt, xs[i], torch.randn(batch, L), 0)
    dt = time.perf_counter() - t0
    return {"value": round(batch * n / dt, 2), "unit": "strain-vectors/s", "cores": threads, "kind": "port",
            "sample": f"oracle train_step (torch-CPU fp32 autograd, reference op order), v0 G={G} H={H} L={L}, "
                      f"{n} steps of {batch} rows of the same synthetic pan-genome matrix after 1 warm-up step, "
                      f"{dt:.1f}s on {threads} threads"}


def gpu_precision_line(mat, G, H, L, B, prec, steps, dev):
    """ms/step and strain-vectors/s of the same C2 step in another GEMM precision (the f32 line
    next to the bf16 headline)."""
    from gm2 import native
    from gm2.model import VAE
    from gm2.trainer import Adam
    torch.manual_seed(0)
    model = VAE(G, H, L, device=dev, precision=prec)
    opt = Adam(model, lr=1e-3)
    ws = model.workspace(prec, B)
    grads = torch.zeros_like(model.params)
    scal = torch.tensor(scalar_table(steps + 1), dtype=torch.float32, device=dev)
    loss = torch.zeros(steps + 1, native.LOSS_SLOTS, dtype=torch.float64, device=dev)
    g = torch.Generator().manual_seed(5)
    rows = torch.randperm(mat.n, generator=g)[:B].to(torch.int32).to(dev)

    def step(i):
        eps = torch.randn(B, L, device=dev)
        native.train_fwd_bwd(ws, native.make_batch(mat.data, mat.ld, rows, B, eps), model.params, grads, model.bn,
                             scal[i], loss[i])
        native.grad_norm(ws, model.params, grads, scal[i], loss[i])
        native.adam_step(ws, model.params, grads, opt.exp_avg, opt.exp_avg_sq, scal[i])
    step(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(1, steps + 1):
        step(i)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ls = loss.cpu().numpy()
    if not np.isfinite(ls[0, :3]).all() or not (ls[:, 0] != 0).all():  # (see main())
        raise RuntimeError("the precision line's first step is non-finite or a step did not run")
    del ws, model, opt, grads
    return {"dtype": "f32" if prec == native.GM2_F32 else "bf16", "ms_per_step": round(dt / steps * 1e3, 3),
            "value": round(B * steps / dt, 1), "unit": "strain-vectors/s", "steps": steps}


# preset hyper-parameters of the loss terms (utils/experiments.py:42-114, trainer.py:193-257):
# KL schedule (type, min, max, T), gene abundance (gamma_start, gamma_end, weight) or None, L1 lambda
PRESET_TERMS = {"v0": (("linear", 0.1, 1.0, 10), None, 0.0),
                "v1": (("linear", 0.1, 1.0, 10), (1.0, 0.1, 1.0), 0.01),
                "v2": (("cosine", 0.0, 1.0, 10), (1.0, 0.1, 1.0), 0.01),
                "v3": (("cosine", 0.1, 1.0, 50), (2.0, 0.1, 1.0), 0.01)}


def scalar_table(nsteps, preset="v0", n_epochs=10000):
    """Per-step scalar table of `preset` at epoch 0 of an n_epochs run, from the host schedule code
    the trainer uses (gm2.loss_components: the KL beta -- linear, or cosine advancing its counter per
    batch -- w * gamma of the gene abundance, lambda of L1)."""
    from gm2 import native
    from gm2.loss_components import GeneAbundanceLoss, KLDivergenceLoss
    (kind, bmin, bmax, T), ab, lam = PRESET_TERMS[preset]
    kl = KLDivergenceLoss(scheduler_type=kind, min_beta=bmin, max_beta=bmax, T=T)
    kl.n_epochs = n_epochs
    ga = None
    if ab is not None:
        ga = GeneAbundanceLoss(gamma_start=ab[0], gamma_end=ab[1], weight=ab[2])
        ga.n_epochs = n_epochs
    tab = np.zeros((nsteps, native.NUM_SCALARS), np.float64)
    for i in range(nsteps):
        t = i + 1
        tab[i, native.S_BETA] = kl.scalars(0)["beta"]
        tab[i, native.S_WGAMMA] = ga.scalars(0)["wgamma"] if ga is not None else 0.0
        tab[i, native.S_LAMBDA] = lam
        tab[i, native.S_MAX_NORM] = 1.0
        tab[i, native.S_NEG_STEP] = -(1e-3 / (1 - 0.9 ** t))
        tab[i, native.S_BC2_SQRT] = math.sqrt(1 - 0.999 ** t)
        tab[i, native.S_ONE_MINUS_B1], tab[i, native.S_BETA2] = 1 - 0.9, 0.999
        tab[i, native.S_ONE_MINUS_B2], tab[i, native.S_ADAM_EPS] = 1 - 0.999, 1e-8
    return tab


def train_leg(a, dev, dist, rank, world, G, H, L, B, strains, prec, seed_base=12345, preset="v0", x=None,
              steps=None, warmup=None):
    """K timed training steps of `preset` (v0 unless given; after W warm-up steps) of `B` rows per
    rank, on a resident synthetic pan-genome shard of `strains` x G per rank (or the given host
    matrix x): forward, fused loss, backward, (bucketed all-reduce when world > 1), clip statistics
    (+ L1), Adam. Returns the max-over-ranks wall time of the K steps, the live-timed output-layer
    loss kernel, and the per-step loss record (every step's losses and gradient norm must be
    finite)."""
    from gm2 import native
    from gm2.data import ResidentMatrix, synthetic_pangenome
    from gm2.ddp import GradSync
    from gm2.model import VAE
    from gm2.trainer import Adam

    K = a.steps if steps is None else steps
    W = a.warmup if warmup is None else warmup
    if x is None:
        x = synthetic_pangenome(strains, G, seed=seed_base + rank)
    strains = x.shape[0]
    mat = ResidentMatrix(x, device=dev)
    torch.manual_seed(0)  # identical init on every rank
    model = VAE(G, H, L, device=dev, precision=prec)
    opt = Adam(model, lr=1e-3)
    ws = model.workspace(prec, B)
    grads = torch.zeros_like(model.params)
    nsteps = W + K
    # per-step scalar table (the preset's schedules at epoch 0 of a 10000-epoch run: v0 beta 0.1, no
    # abundance / L1; v1-v3 add w * gamma and lambda 0.01, v2 / v3 a cosine beta advancing per batch)
    tab = scalar_table(nsteps, preset)
    # one process: grads reach gm2_grad_norm as gm2_train_fwd_bwd wrote them (no all-reduce between)
    tab[:, native.S_NORM_AHEAD] = 1.0 if dist is None else 0.0
    scal = torch.tensor(tab, dtype=torch.float32, device=dev)
    g = torch.Generator().manual_seed(100 + rank)
    rows = torch.cat([torch.randperm(strains, generator=g)[:B] for _ in range(nsteps + 1)]).to(torch.int32).to(dev)
    loss = torch.zeros(nsteps, native.LOSS_SLOTS, dtype=torch.float64, device=dev)
    torch.cuda.manual_seed(1)
    sync = GradSync(dist, model, grads, exchange=a.grad_exchange) if dist is not None else None
    if sync is not None:
        sync.prepare(ws)
    # tuning switches of this workspace only (A/B measurements)
    if a.input_chunks is not None:
        ws.set_option(native.OPT_INPUT_CHUNKS, a.input_chunks)
    if a.grid_cap is not None:
        ws.set_option(native.OPT_GRID_CAP, a.grid_cap)
    # the output layer's Adam update queued and launched beside the next step's hidden layers
    # (bit-identical; the timed region ends with ws.join(), which launches / waits for the last one)
    ws.set_option(native.OPT_DEFER_OUTPUT_ADAM, a.defer_adam if a.defer_adam is not None else 1)
    # gradient-bucket events only where an exchange waits on them (GM2_OPT_GRAD_BUCKETS)
    ws.set_option(native.OPT_GRAD_BUCKETS, 1 if world > 1 else a.grad_buckets)
    if a.recon_tile is not None:
        ws.set_option(native.OPT_RECON_TILE, a.recon_tile)
    # zero-copy rows (gm2_batch.resident): the resident matrix's bf16 rows + target bits, built once
    # before timing, read in place by each step's input-layer GEMMs and loss epilogue (no gather)
    res = mat.operands(prec) if not a.no_zero_copy else None
    # next-batch staging (gm2_batch.next) only under DDP without zero-copy rows, where the gather
    # fills the wait for the input-layer exchange; on one GPU it measured ~30 us/step slower
    # (profiles/r02_prefetch_ab_*)
    prefetch = dist is not None and not a.no_prefetch and res is None

    def step(i):
        eps = torch.randn(B, L, device=dev)
        # the next step's rows are staged during this step's tail (gm2_batch.next; the last timed step
        # stages one batch nobody uses, so the timed region holds K gathers)
        nxt = native.make_batch(mat.data, mat.ld, rows[(i + 1) * B:(i + 2) * B], B, None) if prefetch else None
        batch = native.make_batch(mat.data, mat.ld, rows[i * B:(i + 1) * B], B, eps, next=nxt, resident=res)
        native.train_fwd_bwd(ws, batch, model.params, grads, model.bn, scal[i], loss[i])
        if sync is not None:
            sync.after_backward(ws)  # bucketed SUM all-reduce overlapped with the backward
        native.grad_norm(ws, model.params, grads, scal[i], loss[i])
        native.adam_step(ws, model.params, grads, opt.exp_avg, opt.exp_avg_sq, scal[i])

    torch.cuda.synchronize()
    for i in range(W):
        step(i)
    ws.join()  # (a queued output-layer update runs before the timed region, the timed steps' inside it)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    native.timing_begin(native.KC_RECON_LOSS | (0 if a.no_adam_timing else native.KC_ADAM))
    t0 = time.perf_counter()
    host_s = 0.0
    for i in range(W, nsteps):
        h0 = time.perf_counter()
        step(i)
        host_s += time.perf_counter() - h0
    ws.join()
    torch.cuda.synchronize()
    if a.host_timing:  # (stderr: the host's enqueue time per step, the GPU running asynchronously)
        print(f"host enqueue {1e3 * host_s / max(1, nsteps - W):.3f} ms/step", file=sys.stderr)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    native.timing_end()
    k_ms, k_n = native.timing_class(native.KC_RECON_LOSS)
    a_ms, a_n = native.timing_class(native.KC_ADAM)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    losses = loss.cpu().numpy()
    # every step must have run (its BCE slot written) and be finite: BCE, sum p, KL and the
    # gradient norm of every warm-up and timed step
    if not (losses[:, 0] != 0).all():
        raise RuntimeError("a benchmark step did not run (its loss slot is still zero)")
    bad = ~np.isfinite(losses[:, [0, 1, 2, 4]]).all(axis=1)
    if bad.any():
        raise RuntimeError(f"non-finite loss / gradient norm at step(s) {np.flatnonzero(bad).tolist()}")
    info = {"prefetch": prefetch, "input_chunks": ws.get_option(native.OPT_INPUT_CHUNKS),
            "defer_adam": ws.get_option(native.OPT_DEFER_OUTPUT_ADAM),
            "grad_buckets": ws.get_option(native.OPT_GRAD_BUCKETS),
            "zero_copy": res is not None,
            # the fused L1 + clip + Adam passes: 30 B per parameter per step (read p, g, m, v; write
            # p, m, v and the bf16 / fp32 GEMM shadow), two launches per step (the output layer's deferred)
            "adam": {"ms": a_ms, "launches": a_n, "bytes": 30.0 * model.n_params * (nsteps - W)
                     if prec == native.GM2_BF16 else 32.0 * model.n_params * (nsteps - W)},
            "x": x if (rank == 0 and world == 1) else None, "mat": mat}
    del model, opt, ws, grads, sync
    return elapsed, k_ms, k_n, info


def roofline_entry(a, prec, G, H, B, k_ms, k_n, pmc=True):
    """Output-layer loss GEMM [B,H]x[H,G] + fused BCE/dlogits epilogue against the MFMA roofline:
    achieved = 2*B*H*G FLOP per launch / its average live-timed launch duration (pmc=False: no
    committed PMC pass covers this launch shape -> traffic null)."""
    from gm2 import native
    k_avg_ms = k_ms / max(k_n, 1)
    k_flops = 2.0 * B * H * G
    achieved = k_flops / (k_avg_ms * 1e-3) / 1e12
    peak = PEAK_BF16_TFLOPS if prec == native.GM2_BF16 else PEAK_F32_TFLOPS
    # (the launch's grid: one 512-thread workgroup per 256x256 genes x strains tile)
    grid = ((G + 255) // 256) * ((B + 255) // 256) * 512 if prec == native.GM2_BF16 else None
    traffic, traffic_src = pmc_traffic(a, "k_gemm_recon_loss", grid) if pmc else (None, None)
    return {"bound": "mfma", "kernel": "k_gemm_recon_loss<bf16>" if prec == native.GM2_BF16
            else "k_gemm_recon_loss<f32>", "achieved": round(achieved, 1), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4), "traffic": traffic, "traffic_source": traffic_src,
            "launch_ms": round(k_avg_ms, 4), "launches": k_n, "flops_per_launch": k_flops}


def adam_roofline(a, ad):
    """k_adam_fused against the HBM roofline: algorithmic bytes (30 B per parameter per step in the
    bf16 workspace: read p, g, m, v; write p, m, v and the bf16 GEMM shadow) over the summed live
    duration of its launches (HIP events on each launch's stream; the output layer's update is the
    deferred launch beside the next step's hidden layers). traffic: the committed PMC pass's
    FETCH_SIZE + WRITE_SIZE of the same two launches."""
    if not ad["ms"]:
        return None
    achieved = ad["bytes"] / (ad["ms"] * 1e-3) / 1e9
    tr = [pmc_traffic(a, "k_adam_fused<unsigned short>", g)[0] for g in (3802112, 65536)]
    return {"bound": "hbm", "kernel": "k_adam_fused<bf16>", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
            "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4),
            "traffic": (sum(tr) if all(t is not None for t in tr) else None),
            "bytes_per_step": ad["bytes"] / max(1, ad["launches"] // 2), "launch_ms": round(ad["ms"] / max(ad["launches"], 1), 4),
            "launches": ad["launches"]}


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}: n_gpus must equal the request")
    # (local % device count: lets a 1-GPU box rehearse the N>1 path with GM2_DIST_BACKEND=gloo;
    # torch.cuda.device_count() does not initialise the GPU)
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("GM2_DIST_BACKEND", "nccl")  # nccl = RCCL; gloo only to rehearse
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from gm2 import native

    G, H, L, B = a.genes, a.hidden, a.latent, a.batch
    prec = native.GM2_BF16 if a.precision == "bf16" else native.GM2_F32
    elapsed, k_ms, k_n, info = train_leg(a, dev, dist, rank, world, G, H, L, B, a.strains, prec)
    value = world * B * a.steps / elapsed
    out = {
        "metric": "strain-vectors/sec (train+sample), v0 preset, 1/2/4/8 MI355X vs host CPU",
        "value": round(value, 1), "unit": "strain-vectors/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": a.precision, "data": "synthetic",
        "config": {"workload": "C2: v0 train step (fwd+bwd+clip+Adam), synthetic pan-genome "
                               f"{a.strains}x{G} u8 resident per GPU (+ its bf16 rows / target bits, read in place), "
                               f"batch {B}/GPU",
                   "preset": "v0", "genes": G, "hidden": H, "latent": L, "global_batch": B * world,
                   "parallelism": f"dp{world}",
                   "grad_exchange": (f"{a.grad_exchange} (decoder.9 / encoder.0 weight buckets; rest f32), RCCL "
                                     f"SUM all-reduce overlapped with the backward, input-layer gradient in "
                                     f"{info['input_chunks']} launch(es)")
                   if world > 1 else "none (one GPU)",
                   "input_prefetch": info["prefetch"], "deferred_output_adam": info["defer_adam"],
                   "grad_bucket_events": info["grad_buckets"], "zero_copy_rows": info["zero_copy"]},
        "train_tflops": round(value * train_flops_per_vector(G, H, L) / 1e12, 2),
        "nonfinite_steps": 0,
        # dominant kernel: decoder output layer GEMM [B,H]x[H,G] + fused BCE/abundance/dlogits epilogue
        "roofline": roofline_entry(a, prec, G, H, B, k_ms, k_n),
        # the step's HBM-bound pass: the fused L1 + clip + Adam kernel, bytes over its live launch time
        "roofline_hbm": adam_roofline(a, info["adam"]),
    }
    x = info.pop("x")
    del info
    torch.cuda.empty_cache()
    if not a.no_c5:
        # C5 (configs[4]): v0 on the synthetic 100k x 20k matrix, each rank its 12,500-strain shard
        Gc = 20000
        el5, k5, n5, inf5 = train_leg(a, dev, dist, rank, world, Gc, H, L, B, a.c5_strains, prec, seed_base=777)
        del inf5
        torch.cuda.empty_cache()
        v5 = world * B * a.steps / el5
        out["c5"] = {"workload": f"C5: v0 train step, synthetic {a.c5_strains}x{Gc} u8 shard per GPU (100,000 x "
                                 f"20,000 over 8), batch {B}/GPU", "value": round(v5, 1), "unit": "strain-vectors/s",
                     "n_gpus": world, "ms_per_step": round(el5 / a.steps * 1e3, 3),
                     "train_tflops": round(v5 * train_flops_per_vector(Gc, H, L) / 1e12, 2),
                     "roofline": roofline_entry(a, prec, Gc, H, B, k5, n5)}
    if not a.no_presets:
        # C3 / C4 per-GPU work: the v1, v2 and v3 presets' training step (hidden 512, latent 32, gene
        # abundance + L1 0.01; v2 / v3 with the cosine KL) on the same F4-shaped shard, B rows per GPU
        Hv, Lv = 512, 32
        out["presets"] = {}
        for pv in ("v1", "v2", "v3"):
            elp, kp, np_, infp = train_leg(a, dev, dist, rank, world, G, Hv, Lv, B, a.strains, prec, preset=pv, x=x)
            del infp
            torch.cuda.empty_cache()
            vp = world * B * a.steps / elp
            out["presets"][pv] = {
                "workload": f"{pv} train step (fwd+bwd+clip+L1+Adam, {PRESET_TERMS[pv][0][0]} KL, gene abundance), "
                            f"G={G} H={Hv} L={Lv}, batch {B}/GPU, same synthetic {a.strains}x{G} shard",
                "value": round(vp, 1), "unit": "strain-vectors/s", "n_gpus": world,
                "ms_per_step": round(elp / a.steps * 1e3, 3),
                "train_tflops": round(vp * train_flops_per_vector(G, Hv, Lv) / 1e12, 2),
                "roofline": roofline_entry(a, prec, G, Hv, B, kp, np_, pmc=False)}
    if rank == 0 and world == 1 and not a.no_c1:
        # C1 (configs[0]) on the GPU: the reference's own training batches at F4 width -- v0 at batch 64
        # (C1) and at the CLI default batch 32 (utils/custom_config.py:25) -- one step per batch as
        # trainer.py:109-120 runs it (fwd+bwd+clip+Adam; rows gathered from the resident matrix)
        out["c1_gpu"] = {}
        for bc in (64, 32):
            elc, kc, nc, infc = train_leg(a, dev, None, 0, 1, G, H, L, bc, a.strains, prec, x=x, steps=100, warmup=10)
            del infc
            torch.cuda.empty_cache()
            vc = bc * 100 / elc
            out["c1_gpu"][f"b{bc}"] = {
                "workload": f"v0 train step, G={G} H={H} L={L}, batch {bc}, synthetic {a.strains}x{G} matrix resident",
                "value": round(vc, 1), "unit": "strain-vectors/s", "ms_per_step": round(elc / 100 * 1e3, 4),
                "steps": 100, "train_tflops": round(vc * train_flops_per_vector(G, H, L) / 1e12, 2),
                "roofline": roofline_entry(a, prec, G, H, bc, kc, nc, pmc=False)}
    if rank == 0 and world == 1 and not a.no_f32_line:
        from gm2.data import ResidentMatrix
        other = native.GM2_F32 if prec == native.GM2_BF16 else native.GM2_BF16
        out["precision_line"] = gpu_precision_line(ResidentMatrix(x, device=dev), G, H, L, B, other, 5, dev)
    if not a.no_sample:
        smp = sample_bench(a, dev, dist, rank, world)
        if rank == 0:
            out["sample"] = smp
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(x, G, H, L, a.cpu_seconds, B)
        # C1 (BASELINE.json configs[0]): the reference's CPU plumbing case, v0 at batch 64
        c1 = cpu_baseline(x, G, H, L, min(8.0, a.cpu_seconds / 2), 64)
        out["cpu_baseline_c1"] = {k: c1[k] for k in ("value", "unit", "cores", "kind", "sample")}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def train_v1_checkpoint(a, dev, G, H, L):
    """The sample leg's checkpoint: a v1 model (hidden 512, latent 32, bf16 GEMMs) trained
    a.sample_train_epochs epochs at lr 1e-3 (batch 4096, clip 1.0, L1 0.01, the v1 KL / abundance
    schedules) on the synthetic pan-genome matrix, so the output weights and activations have
    trained scales (the decode's per-tile gate and certified band see realistic logits). Every rank
    trains the same model on the same data (deterministic kernels)."""
    from gm2.data import ResidentMatrix, StrainLoader, synthetic_pangenome
    from gm2.model import VAE
    from gm2.trainer import Adam, StepLR, create_v1_trainer
    from gm2 import native
    torch.manual_seed(11)
    m = VAE(G, H, L, device=dev, precision=native.GM2_BF16)
    opt = Adam(m, lr=1e-3)
    tr = create_v1_trainer(m, opt, StepLR(opt), a.sample_train_epochs, 1.0, 0.01)
    mat = ResidentMatrix(synthetic_pangenome(a.strains, G, seed=4242), device=dev)
    loader = StrainLoader(mat, None, 4096, shuffle=True)
    for ep in range(a.sample_train_epochs):
        tr.train_epoch(loader, ep)
    torch.cuda.synchronize()
    del mat, loader, tr
    torch.cuda.empty_cache()
    return m


def sample_bench(a, dev, dist=None, rank=0, world=1):
    """C3: v1 preset (hidden 512, latent 32) `--mode sample` of a.sample_genomes genomes (1e6 by
    default) in 65,536-genome chunks from a trained v1 checkpoint (train_v1_checkpoint): z ~ N(0, I)
    drawn on the device (extras.py:197), the decode (fp32 hidden layers; the output layer gated per
    256 x 256 tile between the single bf16 product, the bf16x3 split and exact fp32, certified band
    recomputed in fp64) + threshold into packed masks in HBM (gm2_decode_bits), the essential-gene
    counts of
    every genome on the device (gm2_mask_count_groups, a synthetic 300-gene essential table), and
    the packed masks + counts copied to pinned host memory on a second stream (overlapping the next
    chunk's decode). genomes/s = all of that, end to end; the .npy write to disk is excluded.
    world > 1: the genomes are sharded over the ranks (contiguous slices, no collective: z rows are
    independent); genomes/s = all genomes / max-rank time."""
    from gm2 import native
    from gm2.ddp import rank_slice
    from gm2.masks import essential_groups
    from gm2.model import VAE
    G, H, L = a.genes, 512, 32
    torch.manual_seed(0)
    trained = train_v1_checkpoint(a, dev, G, H, L) if a.sample_train_epochs > 0 else None
    m = trained or VAE(G, H, L, device=dev, precision=native.GM2_F32)
    m.eval()
    chunk = 65536
    n_all = a.sample_genomes
    lo, hi = rank_slice(n_all, rank, world)
    n = hi - lo
    ldb = native.packed_row_bytes(G)
    rng = np.random.Generator(np.random.PCG64(3))
    ess = {f"e{i}": [int(p) for p in rng.integers(0, G, size=int(rng.integers(1, 4)))] for i in range(300)}
    offs, pos = essential_groups(ess, G)
    go, po = torch.from_numpy(offs).to(dev), torch.from_numpy(pos).to(dev)
    host_bits = torch.empty(n, ldb, dtype=torch.uint8, pin_memory=True)   # where the masks end up
    host_cnt = torch.empty(n, dtype=torch.int32, pin_memory=True)
    dbits = [torch.empty(chunk, ldb, dtype=torch.uint8, device=dev) for _ in range(2)]
    dcnt = [torch.empty(chunk, dtype=torch.int32, device=dev) for _ in range(2)]
    # the packed masks leave on a.copy_streams copy streams, each a contiguous share of the chunk's rows
    ncs = max(1, a.copy_streams)
    copies = [torch.cuda.Stream(device=dev) for _ in range(ncs)]
    done = [[torch.cuda.Event() for _ in range(ncs)] for _ in range(2)]
    ws = m.workspace(native.GM2_F32, chunk)

    def run(timed):
        z = torch.randn(n, L, device=dev)
        cur = torch.cuda.current_stream(dev)
        for k, s in enumerate(range(0, n, chunk)):
            b = k & 1
            cnt = min(chunk, n - s)
            for ev in done[b]:
                cur.wait_event(ev)  # the copies of the chunk that last used this buffer have finished
            native.decode_bits(ws, m.params, m.bn, z[s:s + cnt], cnt, dbits[b], ldb)
            native.mask_count_groups(dbits[b], cnt, ldb, go, len(offs) - 1, po, dcnt[b])
            for i, cs in enumerate(copies):
                lo, hi = cnt * i // ncs, cnt * (i + 1) // ncs
                cs.wait_stream(cur)
                with torch.cuda.stream(cs):
                    host_bits[s + lo:s + hi].copy_(dbits[b][lo:hi], non_blocking=True)
                    if i == 0:
                        host_cnt[s:s + cnt].copy_(dcnt[b][:cnt], non_blocking=True)
                    done[b][i].record(cs)
        torch.cuda.synchronize()

    # warm-up on one chunk's worth
    native.decode_bits(ws, m.params, m.bn, torch.randn(chunk, L, device=dev), chunk, dbits[0], ldb)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    native.timing_begin(native.KC_MASK)
    st0 = m.decode_stats()
    t0 = time.perf_counter()
    run(True)
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    k_ms, k_n = native.timing_end()
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    gps = n_all / dt
    n_dec = (n + chunk - 1) // chunk
    st = {k: v - st0[k] for k, v in m.decode_stats().items()}
    # per 256 x 256 tile (genomes x genes) the gate ran one bf16 product over the rounded operands
    # (single tier, K = H), the bf16x3 split (K' = 2H, three MFMAs per fragment pair) or, for the
    # blocks whose bound exceeds both, exact fp32 (128 x 128 tiles, four per block); the fractions are
    # shares of the blocks
    blocks = st["single_tiles"] + st["split_tiles"] + st["exact_tiles"] / 4.0
    single_frac = st["single_tiles"] / blocks if blocks else 0.0
    split_frac = st["split_tiles"] / blocks if blocks else 0.0
    exact_frac = max(0.0, 1.0 - single_frac - split_frac)
    bf16 = single_frac + split_frac > 0.5
    prod = 3 if split_frac > single_frac else 1  # products per element of the dominant bf16 tier
    kflops = 2.0 * chunk * H * G * (prod if bf16 else 1)  # executed by one full-chunk launch
    # every output-layer kernel is launched per decode and each tile runs in the one its block's
    # verdict picks: executed FLOPs (1 product per single element, 3 per split element, 1 per exact
    # element) and useful FLOPs (1 per element) over the time of every mask-kernel launch, against
    # the bf16 peak when the bf16 tiers dominate (the exact kernel runs on the fp32 peak)
    ach = 2.0 * n * H * G * (single_frac + 3 * split_frac + exact_frac) / (k_ms * 1e-3) / 1e12
    useful = 2.0 * n * H * G / (k_ms * 1e-3) / 1e12
    peak = PEAK_BF16_TFLOPS if bf16 else PEAK_F32_TFLOPS
    # the packed masks that reached the host are the decode's: spot-check the last chunk on device
    last = (n - 1) // chunk * chunk
    assert torch.equal(host_bits[last:n].to(dev), dbits[((n - 1) // chunk) & 1][:n - last])
    # (the bf16x3 kernel is k_gemm_mask<Cfg<256, ...>, unsigned short, true>, the exact one <..., float>)
    # (the bf16 tiers run in k_gemm_mask_tiered when the single tier is on, else k_gemm_mask<..., true>;
    # the PMC passes decode from an untrained model, tools/prof.sh)
    tiered = ws.get_option(native.OPT_SAMPLE_SINGLE) != 0
    traffic, traffic_src = pmc_traffic(a, ("k_gemm_mask_tiered<Cfg<256" if tiered else "k_gemm_mask<Cfg<256") if bf16
                                       else "k_gemm_mask<Cfg<128",
                                       pattern="r*_pmc_sample_trained.json" if trained is not None else
                                       "r*_pmc_traffic.json")
    return {"genomes_per_s": round(gps, 1), "preset": "v1", "genomes": n_all, "n_gpus": world, "chunk": chunk,
            "checkpoint": (f"v1 trained {a.sample_train_epochs} epochs (lr 1e-3, batch 4096, L1 0.01) on the synthetic "
                           f"{a.strains}x{G} matrix" if trained is not None else "untrained (xavier init)"),
            "single_fraction": round(single_frac, 4), "split_fraction": round(split_frac, 4),
            "single_tiles": st["single_tiles"], "split_tiles": st["split_tiles"], "exact_tiles": st["exact_tiles"],
            "band_elements": st["band_elements"], "band_flips": st["band_flips"], "band_overflow": st["band_overflow"],
            "overflow_tiles": st["overflow_tiles"],
            "dtype": ("bf16 (output layer, rounded operands; fp64 band recompute) + f32 (hidden layers)" if bf16 and prod == 1
                      else "bf16x3 (fp32 split hi/lo, output layer) + f32 (hidden layers)" if bf16 else "f32"),
            "mask_format": "packed bits (numpy packbits, little)", "includes": "z draw, decode, threshold, pack, "
            "essential-gene counts, D2H of packed masks + counts to pinned host memory",
            "decode_tflops": round(gps * decode_flops_per_genome(G, H, L) / 1e12, 2),
            "mean_essential_present": round(float(host_cnt.float().mean()), 2),
            "roofline": {"bound": "mfma", "kernel": ("k_gemm_mask<bf16, 256x256 pp> (K = H, 1 product)" if bf16 and prod == 1
                                                     else "k_gemm_mask<bf16, 256x256 pp> (K' = 2H, 3 products)" if bf16
                                                     else "k_gemm_mask<f32>"), "achieved": round(ach, 2),
                         "peak": peak, "unit": "TFLOP/s", "frac": round(ach / peak, 4),
                         "useful_tflops": round(useful, 2), "useful_frac": round(useful / peak, 4),
                         "flops_per_launch": kflops,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "launch_ms": round(k_ms / max(n_dec, 1), 4), "launches": k_n, "decodes": n_dec}}


if __name__ == "__main__":
    main()
