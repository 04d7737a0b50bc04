"""Data-parallel strain-row training: one process per GPU, torch.distributed (RCCL under the "nccl"
backend on ROCm; gloo for CPU / single-GPU tests). The reference is single-device (main.py:37);
SURVEY.md §8e defines the sharding this module implements.

Semantics:
  * every rank draws the same global batch (same seeds) and runs the contiguous row share
    `rank_slice` of it through the fused step;
  * the gradient buffer is SUM-all-reduced in GM2_GRAD_BUCKETS contiguous buckets, each started on a
    communication stream as soon as libgm2 has finalised it (gm2_wait_grad_bucket: a device-side
    wait on the bucket's event), so the output-layer bucket's exchange runs under the rest of the
    backward and the input-layer weight gradient's four row quarters (GM2_OPT_INPUT_CHUNKS = 4:
    one launch each) are exchanged under the launches that follow them; L1, clip statistics and Adam then run on the reduced gradient, identically on every
    rank (the losses are sum-reductions, so the reduced gradient is the global-batch gradient
    except that train-mode BatchNorm normalises with each rank's own shard statistics, the
    standard non-synchronised DDP BatchNorm);
  * the per-batch loss sums stay on the device and are reduced once per epoch;
  * BatchNorm running statistics are averaged over ranks at the end of every training epoch, so
    validation, sampling and the saved checkpoint see one set of statistics on every rank. The
    running-stat update is linear in the batch statistics, so one average per epoch equals the
    average of per-step averages (up to fp32 rounding);
  * optional SyncBN (enable_sync_bn, VAETrainer(sync_bn=True), main.py --sync-bn): train-mode
    BatchNorm over the GLOBAL batch through 12 fp64 all-reduces per step inside libgm2, so the step
    is the single-device reference's step on the whole batch; running statistics are then identical
    on every rank and are not averaged.
"""
from __future__ import annotations

import os

import torch

from . import native


def get_dist():
    """torch.distributed when a process group of more than one rank is initialised, else None."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist
    return None


def rank_world(dist=None):
    dist = dist if dist is not None else get_dist()
    return (dist.get_rank(), dist.get_world_size()) if dist else (0, 1)


def rank_slice(n, rank, world):
    """Contiguous share [lo, hi) of a global batch of n rows for `rank` of `world`."""
    return (n * rank) // world, (n * (rank + 1)) // world


def rank_share(n, rank, world):
    """Training share [lo, hi) of a global batch of n >= 2 rows: contiguous slices over the first
    min(world, n // 2) ranks, so every active rank holds >= 2 rows (train-mode BatchNorm needs two,
    model.py:67) and every row of the batch is trained, as in the reference (trainer.py:109-120).
    The remaining ranks get an empty share (lo == hi) and contribute zeros to the exchange."""
    active = max(1, min(world, n // 2))
    if rank >= active:
        return n, n
    return (n * rank) // active, (n * (rank + 1)) // active


def train_rows_cap(batch_size, world, sync_bn=False):
    """Rows the training workspace of one rank must hold: the largest share rank_share (or
    rank_slice under SyncBN) can give for any global batch of n <= batch_size rows. With
    n >= 2 world the shares are <= ceil(n / world); below that n // 2 ranks share n rows, i.e. 2 or
    3 each (e.g. a ragged last batch of 3 rows on 16 ranks: one rank gets all 3)."""
    cap = -(-batch_size // world)
    return cap if sync_bn or world <= 1 else max(cap, min(3, batch_size))


def bf16_exchange_sum(dist, x, scratch=None):
    """SUM over the ranks of the fp32 vector x (every rank's own), moved as bf16 and accumulated in
    fp32: each rank rounds its x to bf16 once, sends chunk j to rank j (all-to-all), rank j sums the
    world's chunks IN RANK ORDER in fp32 and rounds that sum to bf16 once, and an all-gather hands
    every rank every chunk. Bytes per rank: 2 x (world-1)/world x 2 B per element, the same as a
    bf16 ring all-reduce; but the error no longer grows with the ring's per-hop bf16 rounding:
        |result - sum_r x_r| <= 2^-8 (1.001 sum_r |x_r| + |sum_r x_r|)   (elementwise, any world)
    (bf16 keeps 8 significant bits, unit roundoff 2^-8: each x_r is rounded once, the fp32 sum adds
    at most world x 2^-24 of sum_r |x_r|, and the sum is rounded once),
    and every rank gets identical values. Returns the reduced vector (fp32, x's device) in x.
    `scratch`: optional dict reused across calls for the bf16 buffers.
    On a GPU the casts and the rank-order sum are libgm2's kernels (gm2_exchange_pack / _ranksum /
    _unpack); host tensors (the CPU gloo tests of the method) take the same arithmetic in torch.
    gloo with device tensors (the one-GPU rehearsal tests) stages the two collectives through host
    memory; RCCL runs them on the device."""
    world = dist.get_world_size()
    n = x.numel()
    c = -(-n // world)
    if x.is_cuda:
        c = -(-c // 8) * 8  # (the kernels take 16-B chunks)
    sc = scratch if scratch is not None else {}
    if sc.get("n", 0) < world * c or sc["send"].device != x.device:
        for k in ("send", "recv", "gath"):
            sc[k] = torch.empty(world * c, dtype=torch.bfloat16, device=x.device)
        sc["n"] = world * c
    send, recv, gath = sc["send"][:world * c], sc["recv"][:world * c], sc["gath"][:world * c]
    dev = x.is_cuda
    if dev:
        native.exchange_pack(x, send)
    else:
        send[:n].copy_(x)
        send[n:].zero_()
    host = dev and dist.get_backend() == "gloo"
    if host:
        hs, hr = send.cpu(), torch.empty(world * c, dtype=torch.bfloat16)
        dist.all_to_all_single(hr, hs)
        recv.copy_(hr)
    else:
        dist.all_to_all_single(recv, send)
    parts = recv.view(world, c)
    if dev:
        mine = sc.setdefault("mine", torch.empty(0, dtype=torch.bfloat16, device=x.device))
        if mine.numel() < c or mine.device != x.device:  # (a scratch dict reused across devices)
            mine = sc["mine"] = torch.empty(c, dtype=torch.bfloat16, device=x.device)
        mine = mine[:c]
        native.exchange_ranksum(recv, world, mine)
    else:
        acc = parts[0].float()
        for r in range(1, world):  # rank order: the same value on every rank, run to run
            acc.add_(parts[r].float())
        mine = acc.to(torch.bfloat16)
    if host:
        hg = [torch.empty(c, dtype=torch.bfloat16) for _ in range(world)]
        dist.all_gather(hg, mine.cpu())
        gath.copy_(torch.cat(hg))
    else:
        dist.all_gather_into_tensor(gath, mine)
    if dev:
        native.exchange_unpack(gath, x)
    else:
        x.copy_(gath[:n])
    return x


class GradSync:
    """Bucketed SUM all-reduce of the flat gradient buffer, overlapped with the backward.

    exchange="f32" (default) all-reduces the fp32 gradient as it is. exchange="bf16" moves the two
    big weight gradients (buckets 0 and 2..5: decoder.9 and encoder.0, ~96 % of the bytes of v0) as
    bf16 with an fp32 accumulation (bf16_exchange_sum: all-to-all, fp32 sum in rank order, all-gather
    -- half the bytes on xGMI, and an error bound independent of the world size); the hidden/BN
    bucket stays fp32. The result is identical on every rank, and clip / L1 / Adam run on it in fp32
    as before."""

    def __init__(self, dist, model, grads, exchange="f32"):
        if exchange not in ("f32", "bf16"):
            raise ValueError(f"gradient exchange {exchange!r}: 'f32' or 'bf16'")
        self.dist = dist
        self.grads = grads
        self.exchange = exchange
        self.scratch = {}
        self.bounds = native.grad_bucket_bounds(native.dims(model.input_dim, model.hidden_dim,
                                                            model.latent_dim, 1))
        self.stream = torch.cuda.Stream(device=grads.device)

    @staticmethod
    def prepare(ws):
        """The training workspace computes the input-layer weight gradient (half the bytes) as four
        launches, so the exchange of its first quarters runs under the GEMM of the later ones
        (bit-identical results). A per-workspace option: nothing else in the process changes."""
        if ws.get_option(native.OPT_INPUT_CHUNKS) != 4:
            ws.set_option(native.OPT_INPUT_CHUNKS, 4)

    def after_backward(self, ws, ran=True):
        """Enqueue the bucket all-reduces behind the backward just launched on workspace `ws`
        (ran=True), or behind whatever the current stream holds (ran=False: this rank contributed
        zeros)."""
        cur = torch.cuda.current_stream(self.grads.device)
        with torch.cuda.stream(self.stream):
            if not ran:
                self.stream.wait_stream(cur)
            for b, (lo, hi) in enumerate(self.bounds):
                if ran:
                    native.wait_grad_bucket(ws, b, self.stream)
                if self.exchange == "bf16" and b != 1:
                    bf16_exchange_sum(self.dist, self.grads[lo:hi], self.scratch)
                else:
                    self.dist.all_reduce(self.grads[lo:hi])
        cur.wait_stream(self.stream)


def enable_sync_bn(dist, ws):
    """SyncBN on a training workspace (gm2.h GM2_OPT_SYNC_BN): train-mode BatchNorm normalises with
    the statistics of the global batch, every rank's rows, as the single-device reference does
    (model.py:67-86), at the price of 12 small fp64 all-reduces (2H + 2 doubles each) per step,
    issued by libgm2 through this torch.distributed collective on the call's stream."""
    if ws.get_option(native.OPT_SYNC_BN) != 1:
        ws.set_option(native.OPT_SYNC_BN, 1)
        ws.set_collective(lambda t: dist.all_reduce(t))


def reduce_loss_rows(dist, rec):
    """SUM over ranks of the per-rank loss sums [BCE, sum p, KL] of every batch row of the epoch's
    loss record (rec [nb][GM2_LOSS_SLOTS] fp64; slots 3-4 are post-reduction values already
    identical on every rank). One contiguous exchange per epoch."""
    part = rec[:, :3].contiguous()
    dist.all_reduce(part)
    rec[:, :3].copy_(part)


def average_running_stats(dist, bn):
    """Mean over ranks of the BatchNorm running statistics ([6][2][H] fp32, contiguous)."""
    dist.all_reduce(bn)
    bn.mul_(1.0 / dist.get_world_size())


def broadcast_model(dist, model, src=0):
    """Every rank starts from rank `src`'s parameters and statistics (the reference's init draws
    from the unseeded global generator, so ranks would otherwise differ)."""
    dist.broadcast(model.params, src)
    dist.broadcast(model.bn, src)
    model.touch()


def gather_rows(dist, local, n_total):
    """Concatenate every rank's contiguous row slice (rank_slice(n_total, r, world)) of a device
    tensor on every rank: one padded all-gather (slices differ by at most one row). Used by the
    sharded `--mode sample` to hand rank 0 the full mask set for the reference's output files."""
    world = dist.get_world_size()
    spans = [rank_slice(n_total, r, world) for r in range(world)]
    cap = max(hi - lo for lo, hi in spans)
    buf = torch.zeros((cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    buf[: local.shape[0]] = local
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    return torch.cat([parts[r][: hi - lo] for r, (lo, hi) in enumerate(spans)])


def shared_seed(dist, src=0):
    """A seed drawn on rank `src` and broadcast, for identical host RNG streams on every rank."""
    t = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64)
    if dist.get_backend() == "nccl":
        t = t.cuda()
    dist.broadcast(t, src)
    return int(t.item())


def init_from_env(backend=None):
    """torchrun entry (main.py): bind this process to LOCAL_RANK's GPU and initialise the process
    group BEFORE any other GPU work. No-op for a single process. Returns the dist module or None."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return None
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    backend = backend or os.environ.get("GM2_DIST_BACKEND", "nccl")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return dist
