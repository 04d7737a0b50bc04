"""ctypes binding of libgm2.so (include/gm2.h) — the only route from the Python host to the GPU.

There is no fallback: if the library is missing or fails to load, every entry point raises.
Device pointers are passed as integers (`tensor.data_ptr()`), the stream as torch's current
HIP stream handle, so launches are ordered with the surrounding torch work.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

# (env GM2_LIB_PATH: another build of the library, for same-box A/Bs of two builds)
LIB_PATH = os.environ.get("GM2_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgm2.so")

GM2_F32 = 0
GM2_BF16 = 1
NUM_PARAMS = 30
NUM_SCALARS = 16
LOSS_SLOTS = 8

# scalar block indices (gm2.h GM2_S_*)
S_BETA, S_WGAMMA, S_LAMBDA, S_NEG_STEP, S_BC2_SQRT, S_MAX_NORM = 0, 1, 2, 3, 4, 5
S_ONE_MINUS_B1, S_BETA2, S_ONE_MINUS_B2, S_ADAM_EPS = 6, 7, 8, 9
S_NORM_AHEAD = 10

EXPORTS = ["gm2_last_error", "gm2_abi_version", "gm2_param_count", "gm2_param_offsets",
           "gm2_workspace_size", "gm2_workspace_init", "gm2_sync_shadows", "gm2_train_fwd_bwd",
           "gm2_grad_norm", "gm2_adam_step", "gm2_eval_forward", "gm2_decode_mask", "gm2_encode", "gm2_forward", "gm2_backward_outputs",
           "gm2_reparameterize", "gm2_packed_row_bytes", "gm2_decode_bits", "gm2_mask_count_groups",
           "gm2_mask_row_offsets", "gm2_mask_compact", "gm2_recon_counts",
           "gm2_gemm", "gm2_grad_bucket_bounds", "gm2_wait_grad_bucket", "gm2_set_option", "gm2_get_option",
           "gm2_workspace_set_option", "gm2_workspace_get_option", "gm2_workspace_release",
           "gm2_workspace_set_collective", "gm2_workspace_join",
           "gm2_resident_layout", "gm2_resident_build",
           "gm2_timing_begin", "gm2_timing_end", "gm2_timing_class", "gm2_workspace_stat",
           "gm2_exchange_pack", "gm2_exchange_ranksum", "gm2_exchange_unpack"]
ABI_VERSION = 6
KC_RECON_LOSS, KC_GEMM_STORE, KC_MASK, KC_ADAM = 1, 2, 4, 8
OPT_GEMM_PP, OPT_SIDE_STREAM, OPT_RECON_TILE, OPT_SMALL_SPLIT, OPT_BN_EPILOGUE, OPT_SMALL_WAVES = 1, 2, 3, 4, 5, 6
OPT_INPUT_CHUNKS, OPT_GRID_CAP, OPT_SYNC_BN, OPT_DEFER_OUTPUT_ADAM = 7, 9, 10, 11
OPT_GRAD_BUCKETS = 15
OPT_SAMPLE_SPLIT = 18
OPT_SAMPLE_SINGLE = 20
OPT_SAMPLE_BAND_CAP, OPT_SAMPLE_SINGLE_BOUND = 21, 22
STAT_SPLIT_DECODES, STAT_EXACT_DECODES, STAT_SPLIT_TILES, STAT_EXACT_TILES = 1, 2, 3, 4
STAT_BAND_ELEMENTS, STAT_BAND_FLIPS, STAT_BAND_OVERFLOW, STAT_SINGLE_TILES = 5, 6, 7, 8
STAT_OVERFLOW_TILES = 9
# the sampling decode's counters by name (gm2.h GM2_STAT_*)
DECODE_STATS = {"split_decodes": STAT_SPLIT_DECODES, "exact_decodes": STAT_EXACT_DECODES,
                "split_tiles": STAT_SPLIT_TILES, "exact_tiles": STAT_EXACT_TILES,
                "band_elements": STAT_BAND_ELEMENTS, "band_flips": STAT_BAND_FLIPS,
                "band_overflow": STAT_BAND_OVERFLOW, "single_tiles": STAT_SINGLE_TILES,
                "overflow_tiles": STAT_OVERFLOW_TILES}
# gm2_allreduce_fn (gm2.h): int (double* buf, int64_t count, void* stream, void* user)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p)


class Dims(C.Structure):
    _fields_ = [("G", C.c_int64), ("H", C.c_int64), ("L", C.c_int64), ("batch_max", C.c_int64)]


class Batch(C.Structure):
    pass


Batch._fields_ = [("data", C.c_void_p), ("ld_data", C.c_int64), ("rows", C.c_void_p), ("n", C.c_int64),
                  ("eps", C.c_void_p), ("next", C.POINTER(Batch)),
                  ("resident", C.c_void_p), ("ld_resident", C.c_int64), ("resident_bits", C.c_void_p),
                  ("ld_resident_bits", C.c_int64), ("resident_rows", C.c_int64), ("resident_prec", C.c_int)]


_lib = None


def lib():
    """Load libgm2.so once; raises (never falls back) when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libgm2.so not built ({LIB_PATH}); run __graft_entry__.build() or "
                           "python genome-minimizer-2_amd/build_native.py")
    L = C.CDLL(LIB_PATH)
    vp, i64, i32, dp = C.c_void_p, C.c_int64, C.c_int, C.POINTER(Dims)
    sig = {
        "gm2_last_error": (C.c_char_p, []),
        "gm2_abi_version": (C.c_int, []),
        "gm2_param_count": (C.c_int, [dp, C.POINTER(C.c_int64)]),
        "gm2_param_offsets": (C.c_int, [dp, C.POINTER(C.c_int64)]),
        "gm2_workspace_size": (C.c_int, [dp, i32, C.POINTER(C.c_size_t)]),
        "gm2_workspace_init": (C.c_int, [dp, i32, vp, C.c_size_t, vp]),
        "gm2_sync_shadows": (C.c_int, [dp, i32, vp, vp, vp]),
        "gm2_train_fwd_bwd": (C.c_int, [dp, i32, C.POINTER(Batch), vp, vp, vp, vp, vp, vp, vp]),
        "gm2_grad_norm": (C.c_int, [dp, i32, vp, vp, vp, vp, vp, vp]),
        "gm2_adam_step": (C.c_int, [dp, i32, vp, vp, vp, vp, vp, vp, vp]),
        "gm2_eval_forward": (C.c_int, [dp, i32, C.POINTER(Batch), vp, vp, vp, vp, vp, vp]),
        "gm2_decode_mask": (C.c_int, [dp, vp, vp, vp, i64, vp, i64, vp, i64, vp, vp]),
        "gm2_encode": (C.c_int, [dp, i32, C.POINTER(Batch), vp, vp, vp, vp, vp, vp]),
        "gm2_forward": (C.c_int, [dp, i32, C.POINTER(Batch), vp, vp, i32, vp, i64, vp, vp, vp, vp]),
        "gm2_backward_outputs": (C.c_int, [dp, i32, C.POINTER(Batch), vp, i32, vp, i64, vp, vp, vp, vp, vp, vp]),
        "gm2_reparameterize": (C.c_int, [i64, vp, vp, vp, vp, vp, vp, vp, vp]),
        "gm2_packed_row_bytes": (C.c_int64, [i64]),
        "gm2_decode_bits": (C.c_int, [dp, vp, vp, vp, i64, vp, i64, vp, i64, vp, vp]),
        "gm2_mask_count_groups": (C.c_int, [vp, i64, i64, vp, i64, vp, vp, vp]),
        "gm2_mask_row_offsets": (C.c_int, [vp, i64, i64, vp, vp, vp]),
        "gm2_mask_compact": (C.c_int, [vp, i64, i64, vp, vp, vp, vp]),
        "gm2_recon_counts": (C.c_int, [dp, i32, C.POINTER(Batch), vp, vp, C.c_float, vp, vp, vp]),
        "gm2_gemm": (C.c_int, [i32, i32, i32, vp, i64, vp, i64, vp, i64, i64, i64, i64, i32, vp, vp]),
        "gm2_grad_bucket_bounds": (C.c_int, [dp, C.POINTER(C.c_int64)]),
        "gm2_wait_grad_bucket": (C.c_int, [vp, i32, vp]),
        "gm2_set_option": (C.c_int, [i32, i32]),
        "gm2_get_option": (C.c_int, [i32, C.POINTER(C.c_int)]),
        "gm2_workspace_set_option": (C.c_int, [vp, i32, i32]),
        "gm2_workspace_get_option": (C.c_int, [vp, i32, C.POINTER(C.c_int)]),
        "gm2_workspace_release": (C.c_int, [vp]),
        "gm2_workspace_set_collective": (C.c_int, [vp, ALLREDUCE_FN, vp]),
        "gm2_workspace_join": (C.c_int, [vp, vp]),
        "gm2_workspace_stat": (C.c_int, [vp, i32, C.POINTER(C.c_int64)]),
        "gm2_resident_layout": (C.c_int, [i64, i64, i32, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                           C.POINTER(C.c_int64), C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]),
        "gm2_resident_build": (C.c_int, [vp, i64, i64, i64, i32, vp, vp, vp]),
        "gm2_exchange_pack": (C.c_int, [vp, i64, vp, i64, vp]),
        "gm2_exchange_ranksum": (C.c_int, [vp, i32, i64, vp, vp]),
        "gm2_exchange_unpack": (C.c_int, [vp, i64, vp, vp]),
        "gm2_timing_begin": (C.c_int, [i32]),
        "gm2_timing_end": (C.c_int, [C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
        "gm2_timing_class": (C.c_int, [i32, C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.gm2_abi_version() != ABI_VERSION:
        raise RuntimeError(f"libgm2 ABI mismatch: library {L.gm2_abi_version()}, binding {ABI_VERSION}")
    _lib = L
    return L


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().gm2_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def dims(G, H, L, batch_max) -> Dims:
    return Dims(int(G), int(H), int(L), int(batch_max))


def param_offsets(G, H, L):
    d = dims(G, H, L, 1)
    off = (C.c_int64 * (NUM_PARAMS + 1))()
    check(lib().gm2_param_offsets(C.byref(d), off), "gm2_param_offsets")
    return list(off)


def workspace_size(d: Dims, prec: int) -> int:
    n = C.c_size_t()
    check(lib().gm2_workspace_size(C.byref(d), prec, C.byref(n)), "gm2_workspace_size")
    return n.value


class Workspace:
    """Caller-owned device scratch of one (dims, precision) geometry, with its own tuning options
    (set_option) and host-side state in libgm2 (released with the buffer).

    `gen` counts the calls that overwrote the workspace's activations (every wrapper below that
    runs a forward, encode, decode or backward on it), so a holder of activations can check that
    nobody has used the workspace since (model.py _Forward)."""

    def __init__(self, d: Dims, prec: int, device):
        self.d, self.prec = d, prec
        self.nbytes = workspace_size(d, prec)
        self.buf = torch.empty(self.nbytes + 256, dtype=torch.uint8, device=device)
        base = self.buf.data_ptr()
        self.off = (-base) % 256
        self.ptr = C.c_void_p(base + self.off)
        self.gen = 0
        check(lib().gm2_workspace_init(C.byref(d), prec, self.ptr, self.nbytes, stream()),
              "gm2_workspace_init")
        self._lib = lib()

    def set_option(self, key: int, value: int):
        """Tuning switch of this workspace only (gm2.h GM2_OPT_*)."""
        check(lib().gm2_workspace_set_option(self.ptr, int(key), int(value)), "gm2_workspace_set_option")

    def get_option(self, key: int) -> int:
        v = C.c_int()
        check(lib().gm2_workspace_get_option(self.ptr, int(key), C.byref(v)), "gm2_workspace_get_option")
        return v.value

    def join(self):
        """Make torch's current stream wait for work this workspace left running on its side
        stream (a deferred output-layer Adam update, GM2_OPT_DEFER_OUTPUT_ADAM)."""
        check(lib().gm2_workspace_join(self.ptr, stream()), "gm2_workspace_join")

    def stat(self, key: int) -> int:
        """A counter of this workspace's host-side state (gm2.h GM2_STAT_*)."""
        v = C.c_int64()
        check(lib().gm2_workspace_stat(self.ptr, int(key), C.byref(v)), "gm2_workspace_stat")
        return int(v.value)

    def set_collective(self, fn):
        """The SUM all-reduce SyncBN calls (gm2_workspace_set_collective): fn(tensor) reduces a
        float64 device tensor (a view of this workspace) in place on torch's current stream, which
        is the stream of the libgm2 call in progress. None removes it."""
        if fn is None:
            self._coll = None
            check(lib().gm2_workspace_set_collective(self.ptr, ALLREDUCE_FN(), None), "gm2_workspace_set_collective")
            return
        base = self.buf.data_ptr()

        def cb(buf, count, strm, user):
            try:
                off = int(buf) - base
                t = self.buf[off: off + 8 * int(count)].view(torch.float64)
                # (the call's stream; NULL = the device's default stream)
                st = torch.cuda.ExternalStream(int(strm), device=self.buf.device) if strm else \
                    torch.cuda.default_stream(self.buf.device)
                with torch.cuda.stream(st):
                    fn(t)
                return 0
            except Exception as e:  # an exception must not cross the C frames
                import sys
                print(f"libgm2 collective failed: {e!r}", file=sys.stderr)
                return 1
        self._coll = ALLREDUCE_FN(cb)  # kept alive as long as the workspace
        check(lib().gm2_workspace_set_collective(self.ptr, self._coll, None), "gm2_workspace_set_collective")

    def __del__(self):
        lb = getattr(self, "_lib", None)
        if lb is not None and getattr(self, "ptr", None) is not None:
            try:
                # the device memory may still be read by queued kernels; the caching allocator
                # reuses it only in stream order, and only the host-side state goes here
                lb.gm2_workspace_release(self.ptr)
            except Exception:
                pass


class ResidentOperands:
    """The resident matrix as GEMM operands (gm2_resident_build): T rows [S + 1 ...][ld] with a zero
    row S and zero pad columns, and their packed target bits [..][ld_bits]; training calls read the
    batch's rows in place through gm2_batch.resident (no per-step gather)."""

    def __init__(self, data, ld_data, S, G, prec):
        ld, ldb, rows = C.c_int64(), C.c_int64(), C.c_int64()
        nb, nbb = C.c_size_t(), C.c_size_t()
        check(lib().gm2_resident_layout(int(S), int(G), prec, C.byref(ld), C.byref(ldb), C.byref(rows), C.byref(nb),
                                        C.byref(nbb)), "gm2_resident_layout")
        dt = torch.float32 if prec == GM2_F32 else torch.bfloat16
        self.rows_t = torch.empty(rows.value, ld.value, dtype=dt, device=data.device)
        self.bits = torch.empty(rows.value, ldb.value, dtype=torch.int32, device=data.device)
        self.ld, self.ld_bits, self.S, self.prec = ld.value, ldb.value, int(S), prec
        check(lib().gm2_resident_build(data.data_ptr(), int(ld_data), int(S), int(G), prec, self.rows_t.data_ptr(),
                                       self.bits.data_ptr(), stream()), "gm2_resident_build")


def make_batch(data, ld, rows, n, eps, next: "Batch | None" = None,
               resident: "ResidentOperands | None" = None) -> Batch:
    """`next` (training only): the batch the following train_fwd_bwd on the same workspace gets; its
    rows are gathered during this step's tail (gm2_batch.next). Keep its tensors unchanged until then.
    `resident` (training only): the same matrix as ResidentOperands, read in place (no gather)."""
    b = Batch(data.data_ptr(), int(ld), None if rows is None else rows.data_ptr(), int(n),
              None if eps is None else eps.data_ptr())
    # the tensors the descriptor points at stay alive as long as it does (a staged `next` batch is
    # matched by address in the following call: its rows must not be freed and reallocated before)
    b._keep = (data, rows, eps)
    if next is not None:
        b.next = C.pointer(next)
        b._keep_next = next
    if resident is not None:
        b.resident = resident.rows_t.data_ptr()
        b.ld_resident = resident.ld
        b.resident_bits = resident.bits.data_ptr()
        b.ld_resident_bits = resident.ld_bits
        b.resident_rows = resident.S
        b.resident_prec = resident.prec
        b._keep_res = resident
    return b


def sync_shadows(ws: Workspace, params):
    check(lib().gm2_sync_shadows(C.byref(ws.d), ws.prec, ptr(params), ws.ptr, stream()), "gm2_sync_shadows")


def train_fwd_bwd(ws: Workspace, batch: Batch, params, grads, bn, scal, loss):
    ws.gen += 1
    check(lib().gm2_train_fwd_bwd(C.byref(ws.d), ws.prec, C.byref(batch), ptr(params), ptr(grads), ptr(bn),
                                  ptr(scal), ptr(loss), ws.ptr, stream()), "gm2_train_fwd_bwd")


def grad_norm(ws: Workspace, params, grads, scal, loss):
    check(lib().gm2_grad_norm(C.byref(ws.d), ws.prec, ptr(params), ptr(grads), ptr(scal), ptr(loss), ws.ptr,
                              stream()), "gm2_grad_norm")


def adam_step(ws: Workspace, params, grads, m, v, scal):
    check(lib().gm2_adam_step(C.byref(ws.d), ws.prec, ptr(params), ptr(grads), ptr(m), ptr(v), ptr(scal), ws.ptr,
                              stream()), "gm2_adam_step")


def eval_forward(ws: Workspace, batch: Batch, params, bn, scal, loss):
    ws.gen += 1
    check(lib().gm2_eval_forward(C.byref(ws.d), ws.prec, C.byref(batch), ptr(params), ptr(bn), ptr(scal),
                                 ptr(loss), ws.ptr, stream()), "gm2_eval_forward")


def decode_mask(ws: Workspace, params, bn, z, n, mask, ld_mask, probs=None, ld_probs=0):
    ws.gen += 1
    check(lib().gm2_decode_mask(C.byref(ws.d), ptr(params), ptr(bn), ptr(z), int(n), ptr(mask), int(ld_mask),
                                ptr(probs), int(ld_probs), ws.ptr, stream()), "gm2_decode_mask")


def encode(ws: Workspace, batch: Batch, params, bn, mu, logvar):
    ws.gen += 1
    check(lib().gm2_encode(C.byref(ws.d), ws.prec, C.byref(batch), ptr(params), ptr(bn), ptr(mu), ptr(logvar),
                           ws.ptr, stream()), "gm2_encode")


def forward(ws: Workspace, batch: Batch, params, bn, train, probs, ld_probs, mu=None, logvar=None):
    ws.gen += 1
    check(lib().gm2_forward(C.byref(ws.d), ws.prec, C.byref(batch), ptr(params), ptr(bn), int(train), ptr(probs),
                            int(ld_probs), ptr(mu), ptr(logvar), ws.ptr, stream()), "gm2_forward")


def backward_outputs(ws: Workspace, batch: Batch, params, train, probs, ld_probs, dprobs, dmu, dlogvar, grads):
    ws.gen += 1
    check(lib().gm2_backward_outputs(C.byref(ws.d), ws.prec, C.byref(batch), ptr(params), int(train), ptr(probs),
                                     int(ld_probs), ptr(dprobs), ptr(dmu), ptr(dlogvar), ptr(grads), ws.ptr,
                                     stream()), "gm2_backward_outputs")


def reparameterize(n, mu, logvar, eps, z, dz=None, dmu=None, dlogvar=None):
    check(lib().gm2_reparameterize(int(n), ptr(mu), ptr(logvar), ptr(eps), ptr(z), ptr(dz), ptr(dmu), ptr(dlogvar),
                                   stream()), "gm2_reparameterize")


def packed_row_bytes(G: int) -> int:
    """Row pitch (bytes) of a packed mask of G genes (gm2.h)."""
    return int(lib().gm2_packed_row_bytes(int(G)))


def decode_bits(ws: Workspace, params, bn, z, n, bits, ld_bits, probs=None, ld_probs=0):
    ws.gen += 1
    check(lib().gm2_decode_bits(C.byref(ws.d), ptr(params), ptr(bn), ptr(z), int(n), ptr(bits), int(ld_bits),
                                ptr(probs), int(ld_probs), ws.ptr, stream()), "gm2_decode_bits")


def mask_count_groups(bits, n, ld_bits, group_offsets, n_groups, positions, counts):
    check(lib().gm2_mask_count_groups(ptr(bits), int(n), int(ld_bits), ptr(group_offsets), int(n_groups),
                                      ptr(positions), ptr(counts), stream()), "gm2_mask_count_groups")


def mask_row_offsets(bits, n, ld_bits, keep_bits, offsets):
    check(lib().gm2_mask_row_offsets(ptr(bits), int(n), int(ld_bits), ptr(keep_bits), ptr(offsets), stream()),
          "gm2_mask_row_offsets")


def mask_compact(bits, n, ld_bits, keep_bits, offsets, indices):
    check(lib().gm2_mask_compact(ptr(bits), int(n), int(ld_bits), ptr(keep_bits), ptr(offsets), ptr(indices),
                                 stream()), "gm2_mask_compact")


def recon_counts(ws: Workspace, batch: Batch, params, bn, threshold, counts):
    ws.gen += 1
    check(lib().gm2_recon_counts(C.byref(ws.d), ws.prec, C.byref(batch), ptr(params), ptr(bn), float(threshold),
                                 ptr(counts), ws.ptr, stream()), "gm2_recon_counts")


def gemm(prec, P, ldp, Q, ldq, Cout, ldc, M, N, K, splits=1, slab=None, p_kmajor=True, q_kmajor=True):
    check(lib().gm2_gemm(prec, int(p_kmajor), int(q_kmajor), ptr(P), ldp, ptr(Q), ldq, ptr(Cout), ldc, M, N, K,
                         splits, ptr(slab), stream()), "gm2_gemm")


GRAD_BUCKETS = 6


def grad_bucket_bounds(d: Dims):
    """[(lo, hi)] element ranges of the flat gradient buffer, in backward completion order."""
    lh = (C.c_int64 * (2 * GRAD_BUCKETS))()
    check(lib().gm2_grad_bucket_bounds(C.byref(d), lh), "gm2_grad_bucket_bounds")
    return [(lh[2 * i], lh[2 * i + 1]) for i in range(GRAD_BUCKETS)]


def wait_grad_bucket(ws: Workspace, bucket: int, stream_obj):
    """Make `stream_obj` (a torch.cuda.Stream) wait until gradient bucket `bucket` of the last
    backward on workspace `ws` is final (device-side wait)."""
    check(lib().gm2_wait_grad_bucket(ws.ptr, int(bucket), C.c_void_p(stream_obj.cuda_stream)), "gm2_wait_grad_bucket")


def exchange_pack(x, out):
    """out[:n] = bf16(x) (RNE), out[n:] = 0 (gm2_exchange_pack; x fp32, out bf16, both on the device)."""
    check(lib().gm2_exchange_pack(ptr(x), x.numel(), ptr(out), out.numel(), stream()), "gm2_exchange_pack")


def exchange_ranksum(parts, world, out):
    """out = bf16(fp32 sum of the `world` chunks of `parts` in rank order) (gm2_exchange_ranksum)."""
    check(lib().gm2_exchange_ranksum(ptr(parts), int(world), out.numel(), ptr(out), stream()), "gm2_exchange_ranksum")


def exchange_unpack(src, x):
    """x = fp32(src[:x.numel()]) (gm2_exchange_unpack)."""
    check(lib().gm2_exchange_unpack(ptr(src), x.numel(), ptr(x), stream()), "gm2_exchange_unpack")


def set_option(key: int, value: int):
    """Process DEFAULT of a tuning switch (gm2.h GM2_OPT_*): what workspaces created afterwards
    start with. To change a live workspace use Workspace.set_option."""
    check(lib().gm2_set_option(int(key), int(value)), "gm2_set_option")


def get_option(key: int) -> int:
    v = C.c_int()
    check(lib().gm2_get_option(int(key), C.byref(v)), "gm2_get_option")
    return v.value


def timing_begin(classes: int):
    check(lib().gm2_timing_begin(int(classes)), "gm2_timing_begin")


def timing_end():
    """(total_ms, launches) of the timed kernel class since timing_begin."""
    ms, n = C.c_double(), C.c_int64()
    check(lib().gm2_timing_end(C.byref(ms), C.byref(n)), "gm2_timing_end")
    return ms.value, n.value


def timing_class(cls: int):
    """(total_ms, launches) of one class of the last timed region (after timing_end)."""
    ms, n = C.c_double(), C.c_int64()
    check(lib().gm2_timing_class(int(cls), C.byref(ms), C.byref(n)), "gm2_timing_class")
    return ms.value, n.value
