// C-ABI of libgm2 (include/gm2.h): workspace layout + the per-step kernel schedule of the VAE
// train / eval / sample hot path. Host-side only; kernels live in gemm.hip and kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <functional>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/gm2.h"
#include "gm2_common.hpp"
#include "gm2_kernels.hpp"

using namespace gm2;

namespace {

thread_local std::string g_err;

#define HIP_OK(x)                                                                                  \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) throw Gm2Error("%s:%d %s: %s", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
  } while (0)

template <typename F>
int guarded(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  } catch (...) {
    g_err = "unknown error";
    return -2;
  }
}

// reference parameter order (model.py:65-91)
enum P {
  E0W, E0B, E1G, E1BT, E3W, E3B, E4G, E4BT, E6W, E6B, E7G, E7BT, MUW, MUB, LVW, LVB,
  D0W, D0B, D1G, D1BT, D3W, D3B, D4G, D4BT, D6W, D6B, D7G, D7BT, D9W, D9B, NP
};
static_assert(NP == GM2_NUM_PARAMS, "param count");

struct Dims {
  int64_t G, H, L, Bm;
  int64_t Gp, Lp, K2L, L2r, Lr;
  int64_t off[NP + 1];
};

// gpad: the padding of the gene axis G. The bf16 workspaces pad it to 256 so that every GEMM with a
// G-wide side (input layer, output layer + loss, their weight gradients) tiles into the 256x256
// kernels (C5's G = 20,000 would otherwise be 20,096 = 78.5 x 256 and fall to the 128-tiles); the
// f32 workspaces (sampling decode, parity) keep 128.
Dims make_dims(const gm2_dims* d, int gpad = kTile) {
  if (!d) throw Gm2Error("null dims");
  Dims x;
  x.G = d->G, x.H = d->H, x.L = d->L;
  if (x.G <= 0 || x.H <= 0 || x.L <= 0 || d->batch_max <= 0) throw Gm2Error("dims must be positive");
  if (x.H % kTile) throw Gm2Error("hidden_dim %lld must be a multiple of 128", (long long)x.H);
  if (256 % x.L) throw Gm2Error("latent_dim %lld must divide 256", (long long)x.L);
  x.Bm = round_up(d->batch_max, kTile);
  x.Gp = round_up(x.G, gpad);
  x.Lp = round_up(x.L, kKPad);
  x.K2L = round_up(2 * x.L, kKPad);
  x.L2r = round_up(2 * x.L, kTile);
  x.Lr = round_up(x.Lp, kTile);
  const int64_t G = x.G, H = x.H, L = x.L;
  const int64_t sz[NP] = {H * G, H, H, H, H * H, H, H, H, H * H, H, H, H, L * H, L, L * H, L,
                          H * L, H, H, H, H * H, H, H, H, H * H, H, H, H, G * H, G};
  x.off[0] = 0;
  for (int i = 0; i < NP; ++i) x.off[i + 1] = x.off[i] + sz[i];
  return x;
}

// ---------------------------------------------------------------------------------------------
// workspace layout (bytes). Everything 256-B aligned. Element size es = 4 (F32) or 2 (BF16).
// ---------------------------------------------------------------------------------------------
// The gated sampling decode's control block (uint32 words, workspace region s3ctl):
//   [0, 16)    cumulative uint64[8] (k_decode_stats; zero from gm2_workspace_init), read by
//              gm2_workspace_stat: split tiles, exact tiles, band elements, band flips, band
//              overflow, decodes with split tiles, decodes without
//   [16, 48)   split-kernel tiles of this call (sharded), [48, 80) exact-kernel tiles
//   [80, 144)  band elements this call put in each list shard, 144 bits its recompute flipped
//   [160, 224) band elements this call put in tile slots (sharded)
//   [224, 256) single-product-kernel tiles of this call
//   [256, ...) block maxima of the row norms: activations (roundup(n, 256) / 256), then weights
// Words [16, 256 + blocks) are zeroed at the start of every gated decode.
struct DecodeCtl {
  static constexpr int kCum = 0, kTilesSplit = 16, kTilesExact = 48, kCounts = 80, kFlips = 80 + kBandShards,
                       kTileFound = 160, kTilesSingle = 160 + kBandShards, kBlk = kTilesSingle + kSplitShards;
  static_assert(kFlips < kTileFound && kBlk == 256, "control block");
};

struct Layout {
  Dims d;
  int prec;
  int64_t es;
  // GEMM shadows (T), natural [out][in] layout, zero-padded: each serves as a K-major operand in
  // the forward GEMM and as an MN-major operand ([K=out][N=in]) in the backward dX GEMM
  int64_t sE0, sE1, sE2, sHD, sD0, sD1, sD2, sD3;
  int64_t X, XB, Y[6], A[6], save[6], HD, Z, dL, slabs, slab_cap, side_slabs, side_cap, dY[6], DA, dH;
  int64_t AT5, dYT0;  // transposed A5 / dY0 [H][Bm]: K-major operands of the dW9 / dWe0 GEMMs
  int64_t bnpart, colpart, colpart_cap, losspart, losspart_cap, klpart, gradpart, clip, scal0, total;
  int64_t colbwd, colbwd_cap;  // per-layer bias-gradient partials of the backward (summed on the side stream)
  int64_t nahdr, nasq;         // norm-ahead header int[4] and per-tile sums of squares (NormAhead)
  int64_t X1, XB1;             // second input slot: the next batch's rows, staged under this step's tail
  int64_t syncb;               // SyncBN all-reduce vector: 2H + 2 doubles
  // gated sampling decode (f32 workspaces; GM2_OPT_SAMPLE_SPLIT): the split activations
  // [roundup(Bm, 256)][2H] and output weights [roundup(G, 256)][2H] (bf16, (hi | lo) per 32 columns),
  // their row norms (s3rn, s3cn), the control block (DecodeCtl), the band list and the split
  // kernel's per-tile band slots (s3tlist [tiles][kBandTileSlots] (row, gene), s3tcount [tiles])
  int64_t s3a, s3w, s3rn, s3cn, s3ctl, s3band, s3tlist, s3tcount;
  int64_t s3a1, s3w1;          // the single-product tier's operands: the hi parts alone, [rows][H] bf16
  // band-list overflow (MaskBand.oflag / olist / ocount, k_band_tile_fix), uint32 words: [0, 2) the
  // cumulative count of recomputed blocks (uint64), [4] this call's block count, [64, 64 + tiles) the
  // per-block flags, then [tiles] the listed block ids. Words [4, 64 + tiles) zeroed per decode.
  int64_t s3ovf;
  static constexpr int kOvfCount = 4, kOvfFlags = 64;
  // u8 masks of the gated decode (gm2_decode_mask): its packed bits [roundup(Bm, 256)][s3ldb], expanded
  // to the caller's rows by one streaming pass (k_expand_bits)
  int64_t s3bits, s3ldb;
  int64_t adamscal;            // scalar block of a queued output-layer Adam update
  int64_t ridx;                // zero-copy rows: int32 [roundup(Bm, 256)] resident-matrix row per batch row
};

#ifdef GM2_DEBUG
// (offset, bytes) of every region the last make_layout on this thread took (gm2_debug_check_layout)
thread_local std::vector<std::pair<int64_t, int64_t>> t_regions;
#endif

Layout make_layout(const gm2_dims* gd, int prec) {
  if (prec != GM2_F32 && prec != GM2_BF16) throw Gm2Error("bad precision %d", prec);
  Layout o;
  o.d = make_dims(gd, prec == GM2_BF16 ? 2 * kTile : kTile);
  o.prec = prec;
  o.es = prec == GM2_F32 ? 4 : 2;
  const Dims& d = o.d;
  int64_t cur = 0;
#ifdef GM2_DEBUG
  t_regions.clear();
#endif
  auto take = [&](int64_t bytes) {
    const int64_t at = cur;
    if (bytes < 0) throw Gm2Error("layout: negative region (%lld bytes)", (long long)bytes);
    cur += round_up(bytes, 256);
#ifdef GM2_DEBUG
    t_regions.emplace_back(at, bytes);
#endif
    return at;
  };
  const int64_t es = o.es, H = d.H, Bm = d.Bm;
  o.sE0 = take(H * d.Gp * es);       // [H][Gp]
  o.sE1 = take(H * H * es);          // [H][H]
  o.sE2 = take(H * H * es);
  o.sHD = take(d.L2r * H * es);      // [L2r][H]: rows 0..L-1 mean_layer, L..2L-1 logvar_layer
  o.sD0 = take(H * d.Lr * es);       // [H][Lr]
  o.sD1 = take(H * H * es);
  o.sD2 = take(H * H * es);
  o.sD3 = take(d.Gp * H * es);       // [Gp][H]
  o.X = take(Bm * d.Gp * es);        // gathered strain rows [Bm][Gp]
  o.XB = take(Bm * (d.Gp / 32) * 4); // row-major bit-packed target [Bm][Gp/32]
  for (int i = 0; i < 6; ++i) {
    o.Y[i] = take(Bm * H * 4);       // pre-BN fp32
    o.A[i] = take(Bm * H * es);      // post-ReLU
    o.save[i] = take(2 * H * 4);     // batch mean / invstd
  }
  o.HD = take(Bm * 2 * d.L * 4);     // mu | logvar fp32
  o.Z = take(Bm * d.Lr * es);        // z [Bm][Lr]
  o.dL = take(Bm * d.Gp * es);       // dL/dlogit [Bm][Gp]
  const int64_t maxN = std::max<int64_t>({H, 2 * d.L, d.Lr, 128});
  o.slab_cap = std::max<int64_t>(1024LL * kTile * kTile, 4 * Bm * maxN);
  o.slabs = take(o.slab_cap * 4);
  // weight-gradient GEMMs run on a side stream: their own split-K scratch, one dY per layer
  o.side_cap = std::max<int64_t>(8LL * H * std::max<int64_t>(H, d.L2r), 1024LL * kTile * kTile);
  o.side_slabs = take(o.side_cap * 4);
  for (int i = 0; i < 6; ++i) o.dY[i] = take(Bm * H * es);
  o.DA = take(Bm * H * 4);           // summed split-K input gradient (fp32)
  o.dH = take(Bm * d.L2r * es);      // d(mu | logvar) [Bm][L2r]
  o.AT5 = take(H * Bm * es);
  o.dYT0 = take(H * Bm * es);
  o.bnpart = take((Bm / kBnRowChunk) * H * 8);
  o.colpart_cap = std::max<int64_t>({(Bm / 64) * d.Gp, (Bm / 64) * H, (Bm / 64) * 2 * d.L});
  o.colpart = take(o.colpart_cap * 4);
  o.losspart_cap = std::max<int64_t>((d.Gp / kTile) * (Bm / kTile) * 2, Bm / 64);
  o.losspart = take(o.losspart_cap * 4);
  o.klpart = take((Bm / kReparamRows) * 4);
  o.gradpart = take(2048 * 2 * 8);
  o.colbwd_cap = std::max<int64_t>((Bm / 64) * std::max<int64_t>(H, 2 * d.L), (Bm / kReparamRows) * 2 * d.L);
  o.colbwd = take(7 * o.colbwd_cap * 4);
  o.nahdr = take(16);
  o.nasq = take(2 * (d.Gp / kTile + 1) * (H / kTile + 1) * 8);
  o.clip = take(64);
  o.scal0 = take(GM2_NUM_SCALARS * 4);
  o.X1 = take(Bm * d.Gp * es);
  o.XB1 = take(Bm * (d.Gp / 32) * 4);
  o.syncb = take((2 * H + 2) * 8);
  const bool split3 = prec == GM2_F32;
  o.s3a = take(split3 ? round_up(Bm, 2 * kTile) * 2 * H * 2 : 0);
  o.s3w = take(split3 ? round_up(d.G, 2 * kTile) * 2 * H * 2 : 0);
  o.s3rn = take(split3 ? round_up(Bm, 2 * kTile) * 4 : 0);
  o.s3cn = take(split3 ? round_up(d.G, 2 * kTile) * 4 : 0);
  o.s3ctl = take(split3 ? (DecodeCtl::kBlk + round_up(Bm, 2 * kTile) / 256 + round_up(d.G, 2 * kTile) / 256) * 4 : 0);
  o.s3band = take(split3 ? (int64_t)kBandShards * kBandShardCap * 8 : 0);
  const int64_t s3tiles = split3 ? (round_up(Bm, 2 * kTile) / 256) * (round_up(d.G, 2 * kTile) / 256) : 0;
  o.s3tlist = take(s3tiles * kBandTileSlots * 8);
  o.s3tcount = take(s3tiles * 4);
  o.s3a1 = take(split3 ? round_up(Bm, 2 * kTile) * H * 2 : 0);
  o.s3w1 = take(split3 ? round_up(d.G, 2 * kTile) * H * 2 : 0);
  o.s3ovf = take(split3 ? (Layout::kOvfFlags + 2 * s3tiles) * 4 : 0);
  o.s3ldb = split3 ? round_up(d.G, 2 * kTile) / 8 : 0;
  o.s3bits = take(split3 ? round_up(Bm, 2 * kTile) * o.s3ldb : 0);
  o.adamscal = take(GM2_NUM_SCALARS * 4);
  o.ridx = take(round_up(Bm, 2 * kTile) * 4);
  o.total = cur;
  return o;
}

struct WsState;

template <typename T>
struct Ctx {
  const Layout& lo;
  char* ws;
  hipStream_t s;
  const Dims& d;
  int64_t slab_off, slab_cap;  // split-K scratch of this stream
  int64_t xo, xbo;             // input slot of this call: gathered rows X [Bm][Gp] (T), target bits
  WsState* st;                 // host-side state of the workspace
  // zero-copy rows (gm2_batch.resident, training calls): the input layer's GEMMs and the loss
  // epilogue read the resident matrix's rows through ridx [roundup(Bm, 256)] instead of X / XB
  const int32_t* ridx = nullptr;
  const T* xres = nullptr;
  int64_t ld_xres = 0;
  const uint32_t* xbres = nullptr;
  int64_t ld_xbres = 0;
  int64_t res_rows = 0;  // rows of the resident operands (their zero row included): bounds of ridx
  Ctx(const Layout& l, void* w, void* strm, WsState* state = nullptr)
      : lo(l), ws((char*)w), s((hipStream_t)strm), d(l.d), slab_off(l.slabs), slab_cap(l.slab_cap), xo(l.X),
        xbo(l.XB), st(state) {}
  Ctx side(hipStream_t strm) const {
    Ctx c(lo, ws, strm, st);
    c.slab_off = lo.side_slabs;
    c.slab_cap = lo.side_cap;
    c.xo = xo;
    c.xbo = xbo;
    c.ridx = ridx;
    c.xres = xres;
    c.ld_xres = ld_xres;
    c.xbres = xbres;
    c.ld_xbres = ld_xbres;
    c.res_rows = res_rows;
    return c;
  }
  T* t(int64_t off) const { return (T*)(ws + off); }
  float* f(int64_t off) const { return (float*)(ws + off); }
};

// ---------------------------------------------------------------------------------------------
// Host-side state of one workspace (keyed by its device address; created by gm2_workspace_init,
// dropped by gm2_workspace_release). Nothing here is shared between workspaces: two models, or a
// training and a sampling workspace, in one process keep their own options, side stream, gradient
// bucket events and staged input slot. One workspace is used from one host thread at a time.
//
//  * side stream for the weight-gradient GEMMs (fork/join through events; capture-safe), created
//    on first use; GM2_OPT_SIDE_STREAM = 0 keeps everything on the caller's stream.
//  * gradient buckets (data-parallel exchange): ranges of the flat gradient buffer in the order the
//    backward finalises them, each with an event recorded when its last gradient is written
//    (gm2_grad_bucket_bounds / gm2_wait_grad_bucket)
//      0: decoder.9.weight, decoder.9.bias      (output layer: first off the backward)
//      1: encoder.0.bias .. decoder.7.bias      (every hidden / head / BN tensor)
//      2..5: encoder.0.weight row quarters      (input layer: the last weight-gradient GEMM)
//  * the input-slot stage of gm2_batch.next (SlotState below).
// ---------------------------------------------------------------------------------------------
// Per-workspace input-slot state. A training call whose batch carries `next` gathers next's rows
// into the other slot during its own tail; the following training call finds them there (same
// data / ld / rows / n) and starts straight at the input-layer GEMM. Every other call that uses an
// input slot first waits for a pending stage and drops it (it writes slot 0).
struct SlotState {
  bool staged = false;
  int slot = 0;  // slot of the staged batch
  const uint8_t* data = nullptr;
  int64_t ld = 0, n = 0, total = 0;
  const int32_t* rows = nullptr;
  int prec = -1;
};

// Events that only order this device's own streams (fork / join ring, staged input slot, deferred
// update) release at device scope: a system-scope release writes the L2 back at every fork of the
// backward (measured ~7 us of idle main stream per fork). The gradient-bucket events keep the
// system-scope release (a collective's peers may read the buffer). Env GM2_EVENT_FENCE=system
// restores it everywhere (A/B).
unsigned order_event_flags() {
  static const unsigned f = [] {
    const char* e = std::getenv("GM2_EVENT_FENCE");
    return (e && std::string(e) == "system") ? (unsigned)hipEventDisableTiming
                                             : (unsigned)(hipEventDisableTiming | hipEventReleaseToDevice);
  }();
  return f;
}

struct WsState {
  Options opt;
  int dev = -1;
  hipStream_t side = nullptr;
  std::vector<hipEvent_t> ev;  // fork/join ring
  size_t next = 0;
  hipEvent_t bucket[GM2_GRAD_BUCKETS] = {};
  int bucket_ev[GM2_GRAD_BUCKETS] = {0, 1, 2, 3, 4, 5};  // the event that marks bucket b final
  bool recorded = false;  // a training backward has recorded the bucket events
  SlotState slot;
  hipEvent_t slot_done = nullptr;
  gm2_allreduce_fn coll = nullptr;  // SyncBN's all-reduce (gm2_workspace_set_collective)
  void* coll_user = nullptr;
  hipEvent_t adam9_done = nullptr;  // a deferred output-layer Adam update (GM2_OPT_DEFER_OUTPUT_ADAM)
  bool adam9_pending = false;       // launched on the side stream, not yet joined
  int cus = 0;                      // compute units of dev
  int64_t exact_decodes = 0;        // decodes the host sent to the exact-fp32 kernel alone (probs requests,
                                    // GM2_OPT_SAMPLE_SPLIT = 0, preconditions): GM2_STAT_EXACT_DECODES
  const unsigned long long* decode_cum = nullptr;  // the gated decodes' cumulative device counters (DecodeCtl)
  const unsigned long long* decode_ovf = nullptr;  // their cumulative count of overflow-recomputed blocks
  // the queued (not yet launched) output-layer update: launched by kick() beside the next training
  // call's hidden layers, or by join() on the joining stream
  struct QueuedAdam {
    bool queued = false;
    int prec = 0;
    TensorTable tt{};
    const float* g = nullptr;
    float *p = nullptr, *m = nullptr, *v = nullptr;
    const float *scal = nullptr, *clip = nullptr;
  } qadam;

  void create() {
    HIP_OK(hipGetDevice(&dev));
    HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    for (auto& e : bucket) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&slot_done, order_event_flags()));
    HIP_OK(hipEventCreateWithFlags(&adam9_done, order_event_flags()));
  }
  void destroy() {
    if (side) (void)hipStreamDestroy(side);
    for (auto e : ev) (void)hipEventDestroy(e);
    for (auto e : bucket)
      if (e) (void)hipEventDestroy(e);
    if (slot_done) (void)hipEventDestroy(slot_done);
    if (adam9_done) (void)hipEventDestroy(adam9_done);
    side = nullptr;
    ev.clear();
  }
  // the side stream when GM2_OPT_SIDE_STREAM is on (created on first use), else nullptr
  hipStream_t side_stream() {
    if (!opt.side_stream) return nullptr;
    if (!side) {
      HIP_OK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
      if (ev.empty()) {
        ev.resize(64);
        for (auto& e : ev) HIP_OK(hipEventCreateWithFlags(&e, order_event_flags()));
      }
    }
    return side;
  }
  void launch_queued(hipStream_t s, int max_grid = 0) {
    QueuedAdam& q = qadam;
    if (q.prec == GM2_F32) launch_adam_fused<float>(q.tt, q.g, q.p, q.m, q.v, q.scal, q.clip, s, max_grid);
    else launch_adam_fused<bf16_t>(q.tt, q.g, q.p, q.m, q.v, q.scal, q.clip, s, max_grid);
    q.queued = false;
  }
  // a training call's forward, after its input-layer GEMM: start the queued output-layer update on
  // the side stream (ordered after everything on `s` so far)
  void kick(hipStream_t s) {
    if (!qadam.queued) return;
    const hipStream_t sd = side_stream();
    if (!sd) {
      launch_queued(s);
      return;
    }
    order(s, sd);
    // a few workgroups per CU, looping over the blocks: room stays for the hidden layers' GEMM
    // workgroups (an uncapped grid fills every CU and serialises them behind it)
    launch_queued(sd, std::max(1, opt.defer_adam) * std::max(1, cus));
    HIP_OK(hipEventRecord(adam9_done, sd));
    adam9_pending = true;
  }
  // make `s` see a deferred output-layer update: a queued one is launched on `s`, a running one
  // waited for
  void join(hipStream_t s) {
    if (qadam.queued) launch_queued(s);
    if (adam9_pending) HIP_OK(hipStreamWaitEvent(s, adam9_done, 0));
    adam9_pending = false;
  }
  // SyncBN: SUM-all-reduce `count` doubles at device pointer `buf` across the ranks, on `s`
  void allreduce(double* buf, int64_t count, hipStream_t s) {
    if (!coll) throw Gm2Error("GM2_OPT_SYNC_BN needs a collective (gm2_workspace_set_collective)");
    const int rc = coll(buf, count, (void*)s, coll_user);
    if (rc != 0) throw Gm2Error("SyncBN all-reduce failed (%d)", rc);
  }
  // make `to` wait for everything enqueued on `from` so far
  void order(hipStream_t from, hipStream_t to) {
    hipEvent_t e = ev[next++ % ev.size()];
    HIP_OK(hipEventRecord(e, from));
    HIP_OK(hipStreamWaitEvent(to, e, 0));
  }
};

std::mutex& ws_mutex() {
  static std::mutex mu;
  return mu;
}
std::map<void*, std::unique_ptr<WsState>>& ws_map() {
  static std::map<void*, std::unique_ptr<WsState>> m;
  return m;
}

// the state of `ws`; a workspace that was never initialised through gm2_workspace_init (or was
// released) is an error
WsState& ws_state(void* ws) {
  std::lock_guard<std::mutex> lk(ws_mutex());
  auto it = ws_map().find(ws);
  if (it == ws_map().end()) throw Gm2Error("workspace %p is not initialised (gm2_workspace_init)", ws);
  return *it->second;
}

// (re)initialise the state of `ws`: process-default options, no stage, fresh events
WsState& ws_reset(void* ws) {
  std::lock_guard<std::mutex> lk(ws_mutex());
  auto& slot = ws_map()[ws];
  if (slot) slot->destroy();
  slot.reset(new WsState());
  slot->opt = default_options();
  slot->create();
  return *slot;
}

// true: a queued output-layer update was discarded (gm2_workspace_release then returns 1)
bool ws_release(void* ws) {
  std::lock_guard<std::mutex> lk(ws_mutex());
  auto it = ws_map().find(ws);
  if (it == ws_map().end()) return false;
  WsState& st = *it->second;
  const bool dropped = st.qadam.queued;
  // A still-QUEUED output-layer update is dropped, not launched: release can run at garbage-collection
  // time, after the parameter / moment buffers it would write were freed (callers join with
  // gm2_workspace_join before releasing, as gm2.h says; the Python host does). A RUNNING one is
  // waited for: it reads its scalar block from the workspace memory about to be freed.
  st.qadam.queued = false;
  if (st.adam9_pending) {  // (launched on the side stream)
    if (st.side) HIP_OK(hipStreamSynchronize(st.side));
    else HIP_OK(hipEventSynchronize(st.adam9_done));
    st.adam9_pending = false;
  }
  st.destroy();
  ws_map().erase(it);
  return dropped;
}

// first row of quarter q (0..4) of the input-layer weight gradient [H][G]
int64_t input_quarter_row(const Dims& d, int q) { return (d.H * q) / 4; }

void bucket_bounds(const Dims& d, int64_t* lh) {
  lh[0] = d.off[D9W], lh[1] = d.off[NP];
  lh[2] = d.off[E0B], lh[3] = d.off[D9W];
  for (int q = 0; q < 4; ++q) {
    lh[4 + 2 * q] = input_quarter_row(d, q) * d.G;
    lh[5 + 2 * q] = input_quarter_row(d, q + 1) * d.G;
  }
}

// GEMM into the fp32 slab scratch (split-K slices summed by the consumer). Returns #slabs.
template <typename T>
int gemm_to_slabs(const Ctx<T>& c, const T* P, int64_t ldp, int Mp, const T* Q, int64_t ldq, int Np, int M, int N,
                  int K, int64_t ldc, int pk = 1, int qk = 1, const int32_t* prow = nullptr) {
  GemmArgs<T> g{P, ldp, Q, ldq, M, N, K, Mp, Np, 0, pk, qk};
  g.prow = prow;
  if (prow) g.idx_lim = c.res_rows;
  const int64_t slab = (int64_t)Mp * ldc;
  // (the plan's split count, at most what the stream's slab scratch holds)
  const int S = (int)std::min<int64_t>(plan_gemm<T>(g).splits, c.slab_cap / std::max<int64_t>(slab, 1));
  if (S < 1) throw Gm2Error("slab capacity exceeded");
  return launch_gemm_store<T>(g, S, c.f(c.slab_off), nullptr, 0, ldc, slab, nullptr, c.s);
}

// GEMM into C0/C1 (fp32, row split at msplit). Launches with too few tiles to fill the chip are
// split over K into slabs and summed by k_slab_sum (deterministic order).
template <typename T>
void gemm_to(const Ctx<T>& c, const T* P, int64_t ldp, int Mp, const T* Q, int64_t ldq, int Np, int M, int N, int K,
             float* C0, float* C1, int msplit, int64_t ldc, int pk = 1, int qk = 1, const int32_t* qrow = nullptr) {
  GemmArgs<T> g{P, ldp, Q, ldq, M, N, K, Mp, Np, 0, pk, qk};
  g.qrow = qrow;
  if (qrow) g.idx_lim = c.res_rows;
  int S = plan_gemm<T>(g).splits;
  const int64_t slab = round_up((int64_t)M * N, 4);
  if ((int64_t)S * slab > c.slab_cap) S = 1;
  if (S <= 1) {
    launch_gemm_store<T>(g, 1, C0, C1, msplit, ldc, 0, nullptr, c.s);
    return;
  }
  S = launch_gemm_store<T>(g, S, c.f(c.slab_off), nullptr, 0, N, slab, nullptr, c.s);
  launch_slab_sum(c.f(c.slab_off), S, slab, M, N, C0, C1, C1 ? msplit : M, ldc, c.s);
}

// The two big weight-gradient GEMMs of the backward (output layer dW9, stored transposed; input
// layer dWe0). When both are one K pass (`direct`) their epilogues also write per-tile sums of
// squares, [sq9 | sq0] in the norm-ahead area, so gm2_grad_norm need not re-read 2 x H x G floats.
template <typename T>
struct BigGrads {
  GemmArgs<T> g9, g0;
  bool direct;
  int n9, n0;
};
// the input-layer weight gradient as four row-quarter launches (GM2_OPT_INPUT_CHUNKS = 4): only
// when each quarter is whole 256-row tiles of a one-pass plan, like the full launch
template <typename T>
bool input_chunked(const BigGrads<T>& r, int H) {
  if (opts().input_chunks != 4 || H % 1024) return false;
  const GemmPlan p = plan_gemm<T>(r.g0);
  return p.splits == 1 && p.tile == 256;
}

template <typename T>
BigGrads<T> big_grads(const Ctx<T>& c, int Bp) {
  const Layout& l = c.lo;
  const int H = (int)c.d.H, G = (int)c.d.G, Gp = (int)c.d.Gp;
  BigGrads<T> r{{c.t(l.AT5), Bp, c.t(l.dL), Gp, H, G, Bp, H, Gp, 0, 1, 0},
                {c.t(l.dYT0), Bp, c.t(c.xo), Gp, H, G, Bp, H, Gp, 0, 1, 0}, false, 0, 0};
  if (c.ridx) {  // zero-copy rows: X's rows are the resident matrix's, through ridx
    r.g0.Q = c.xres;
    r.g0.ldq = c.ld_xres;
    r.g0.qrow = c.ridx;
    r.g0.idx_lim = c.res_rows;
  }
  r.direct = plan_gemm<T>(r.g9).splits == 1 && plan_gemm<T>(r.g0).splits == 1;
  r.n9 = gemm_tiles<T>(r.g9);
  r.n0 = gemm_tiles<T>(r.g0);
  if ((int64_t)(r.n9 + r.n0) > 2 * (c.d.Gp / kTile + 1) * (c.d.H / kTile + 1)) r.direct = false;
  if (input_chunked(r, (int)c.d.H)) r.direct = false;  // the quarter launches take no clip statistics
  return r;
}

// the 6 BatchNorm blocks: (linear weight, linear bias, bn gamma, bn beta)
const int kBlk[6][4] = {{E0W, E0B, E1G, E1BT}, {E3W, E3B, E4G, E4BT}, {E6W, E6B, E7G, E7BT},
                        {D0W, D0B, D1G, D1BT}, {D3W, D3B, D4G, D4BT}, {D6W, D6B, D7G, D7BT}};

// Pre-BatchNorm Linear: Y = in . W^T + bias (fp32 [Bp][H]) and, when `stats`, the per-128-row
// chunk (mean, M2) partials of Y -> part. One launch when the GEMM plan is a single pass of 128-row
// tiles (statistics in the store epilogue); otherwise split-K slabs + k_bn_fwd_partial.
template <typename T>
void linear_pre_bn(const Ctx<T>& c, const T* in, int64_t ldin, int Bp, const T* W, int64_t ldw, int B, int H, int K,
                   const float* bias, float* Y, float* part, bool stats, const int32_t* prow = nullptr) {
  GemmArgs<T> g{in, ldin, W, ldw, B, H, K, Bp, H, 0};
  StoreEpi bn;
  bn.mode = stats ? 1 : 0;
  bn.part = (float2*)part;
  bn.ldp = H;
  if (!prow && launch_gemm_bn<T>(g, Y, H, bias, bn, c.s)) return;
  const int S = gemm_to_slabs<T>(c, in, ldin, Bp, W, ldw, H, B, H, K, H, 1, 1, prow);
  launch_bn_fwd_partial(c.f(c.slab_off), S, (int64_t)Bp * H, H, bias, B, H, Y, part, c.s);
}

// Tensor tables. kind 0: the 9 Linear weights with their natural-layout shadow (tile0 counts
// 64x64 tiles; fp32 -> shadow sync). kind 1: all 30 parameters in reference order, weights with
// their shadow (tile0 counts 4096-element blocks; fused Adam writes the shadow).
template <typename T>
TensorTable make_table(const Ctx<T>& c, int kind = 0) {
  const Dims& d = c.d;
  const Layout& l = c.lo;
  TensorTable tt{};
  auto tiles_of = [&](const TensorDesc& e) {
    return kind == 1 ? (e.rows * e.cols + 4095) / 4096 : ((e.rows + 63) / 64) * ((e.cols + 63) / 64);
  };
  auto add = [&](int pi, int64_t rows, int64_t cols, int64_t sh, int64_t sld, int64_t srow0) {
    TensorDesc& e = tt.t[tt.n];
    e.off = d.off[pi];
    e.rows = rows;
    e.cols = cols;
    e.shadow = sh >= 0 ? (void*)(c.ws + sh) : nullptr;
    e.sld = sld;
    e.srow0 = srow0;
    e.shadowT = nullptr;
    e.tld = 0;
    e.tile0 = tt.n == 0 ? 0 : tt.t[tt.n - 1].tile0 + tiles_of(tt.t[tt.n - 1]);
    tt.n++;
  };
  const int64_t H = d.H, G = d.G, L = d.L;
  auto vec = [&](int pi, int64_t n) {
    if (kind == 1) add(pi, 1, n, -1, 0, 0);
  };
  add(E0W, H, G, l.sE0, d.Gp, 0);
  vec(E0B, H); vec(E1G, H); vec(E1BT, H);
  add(E3W, H, H, l.sE1, H, 0);
  vec(E3B, H); vec(E4G, H); vec(E4BT, H);
  add(E6W, H, H, l.sE2, H, 0);
  vec(E6B, H); vec(E7G, H); vec(E7BT, H);
  add(MUW, L, H, l.sHD, H, 0);
  vec(MUB, L);
  add(LVW, L, H, l.sHD, H, L);
  vec(LVB, L);
  add(D0W, H, L, l.sD0, d.Lr, 0);
  vec(D0B, H); vec(D1G, H); vec(D1BT, H);
  add(D3W, H, H, l.sD1, H, 0);
  vec(D3B, H); vec(D4G, H); vec(D4BT, H);
  add(D6W, H, H, l.sD2, H, 0);
  vec(D6B, H); vec(D7G, H); vec(D7BT, H);
  add(D9W, G, H, l.sD3, H, 0);
  vec(D9B, G);
  return tt;
}

// the resident matrix rows of a batch: 16-B aligned rows of at least roundup(G, 128) bytes (gm2.h)
void check_batch_data(const gm2_batch* b, const Dims& d, const char* what) {
  if (!b->data) throw Gm2Error("%s: null data", what);
  if (b->ld_data % 16 || b->ld_data < round_up(d.G, kTile) || ((uintptr_t)b->data & 15))
    throw Gm2Error("%s: data rows must be 16-B aligned with ld_data (%lld) a multiple of 16 and >= roundup(G, 128)",
                   what, (long long)b->ld_data);
}

// entries [lo, hi) of a kind-1 table, block indices re-based to 0 (a launch over that subset)
TensorTable table_range(const TensorTable& tt, int lo, int hi) {
  TensorTable r{};
  const int64_t base = tt.t[lo].tile0;
  for (int i = lo; i < hi; ++i) {
    r.t[r.n] = tt.t[i];
    r.t[r.n].tile0 -= base;
    r.n++;
  }
  return r;
}

// ---------------------------------------------------------------------------------------------
// forward (train or eval). Fills A_l (+A_l^T when train), Y_l, save_l, HD, Z, ZT and runs the
// fused reconstruction-loss epilogue (dL, dL^T when with_grad).
// ---------------------------------------------------------------------------------------------
template <typename T>
void forward(const Ctx<T>& c, const gm2_batch* b, const float* prm, float* bn, int train, int with_grad,
             const float* scal, double* loss, float* grads, float* probs = nullptr, int64_t ld_probs = 0,
             int* counts = nullptr, float thr = 0.5f, bool norm_hdr = false, bool staged = false,
             std::function<void(hipStream_t)>* defer_tail = nullptr) {
  const Dims& d = c.d;
  const Layout& l = c.lo;
  const int B = (int)b->n;
  if (B <= 0 || B > d.Bm) throw Gm2Error("batch rows %d outside (0, batch_max=%lld]", B, (long long)d.Bm);
  const bool sync = train && c.st && c.st->opt.sync_bn;
  // (SyncBN: the batch statistics span every rank's rows, so one row here is fine)
  if (train && B < 2 && !sync) throw Gm2Error("Expected more than 1 value per channel when training (batch of 1)");
  check_batch_data(b, d, "batch");
  double* syncb = (double*)(c.ws + l.syncb);
  const int Bp = (int)round_up(B, kTile);
  const int H = (int)d.H, L = (int)d.L;
  // 1) strain rows -> X [Bp][Gp] (T) + bit-packed target (unless a previous training call staged
  // them, or the call reads the resident matrix's rows in place: c.ridx)
  if (c.ridx)
    launch_resident_rows(b->rows, B, (int)round_up(d.Bm, 2 * kTile), b->resident_rows, const_cast<int32_t*>(c.ridx),
                         c.s);
  else if (!staged)
    launch_gather_rows<T>(b->data, b->ld_data, b->rows, B, (int)d.G, c.t(c.xo), d.Gp, (int)d.Gp, Bp,
                          (uint32_t*)(c.ws + c.xbo), d.Gp / 32, c.s);
  // 2) encoder blocks, heads + reparameterisation, decoder blocks (all NT GEMMs)
  const T* in = c.ridx ? c.xres : c.t(c.xo);
  int64_t ldin = c.ridx ? c.ld_xres : d.Gp;
  int Kin = (int)d.Gp;
  const int64_t shadow_in[6] = {l.sE0, l.sE1, l.sE2, l.sD0, l.sD1, l.sD2};
  for (int i = 0; i < 6; ++i) {
    if (i == 3) {
      const int S = gemm_to_slabs<T>(c, c.t(l.A[2]), H, Bp, c.t(l.sHD), H, (int)d.L2r, B, 2 * L, H, 2 * L);
      launch_reparam<T>(c.f(l.slabs), S, (int64_t)Bp * 2 * L, L, prm + d.off[MUB], prm + d.off[LVB], b->eps, B, Bp,
                        c.f(l.HD), c.t(l.Z), d.Lr, nullptr, 0, 0, c.f(l.klpart), c.s);
      in = c.t(l.Z);
      ldin = d.Lr;
      Kin = (int)d.Lp;
    }
    linear_pre_bn<T>(c, in, ldin, Bp, c.t(shadow_in[i]), i == 3 ? d.Lr : Kin, B, H, Kin, prm + d.off[kBlk[i][1]],
                     c.f(l.Y[i]), c.f(l.bnpart), train != 0, i == 0 ? c.ridx : nullptr);
    // a queued output-layer Adam update of the previous step starts here, beside the hidden layers
    // (HBM-bound next to latency-bound small GEMMs; the gather and the input-layer GEMM before this
    // point leave it nothing: one is HBM-bound too, the other holds every CU's registers)
    if (i == 0 && c.st) c.st->kick(c.s);
    if (sync) {  // SyncBN: this rank's column sums -> all-reduce -> the global batch's statistics
      launch_bn_sync_pack(c.f(l.bnpart), B, H, 0, syncb, c.s);
      c.st->allreduce(syncb, 2 * H + 2, c.s);
    }
    launch_bn_fwd_apply<T>(c.f(l.Y[i]), H, c.f(l.bnpart), B, Bp, H, train, prm + d.off[kBlk[i][2]],
                           prm + d.off[kBlk[i][3]], bn + (int64_t)i * 2 * H, bn + (int64_t)i * 2 * H + H,
                           c.f(l.save[i]), c.t(l.A[i]), c.s, sync ? syncb : nullptr);
    in = c.t(l.A[i]);
    ldin = H;
    Kin = H;
  }
  if (c.st) c.st->join(c.s);  // (a deferred output-layer update must be complete before the output layer)
  if (probs || counts) {  // 3') VAE.forward: p = sigmoid(logits) (model.py:89-90) and / or the
                          // per-strain (TP, FP, FN) of (p > thr) vs the strain's genes; no loss
    GemmArgs<T> g{c.t(l.A[5]), H, c.t(l.sD3), H, B, (int)d.G, H, Bp, (int)d.Gp, 0};
    launch_gemm_mask<T>(g, prm + d.off[D9B], nullptr, 0, probs, ld_probs, c.s, nullptr, 0, counts,
                        (const uint32_t*)(c.ws + c.xbo), d.Gp / 32, thr);
    return;
  }
  // 3) output layer + reconstruction loss (+ dlogits), computed as logit^T: genes x strains. A
  // deferred output-layer Adam update of the previous step (side stream) must be complete here.
  if (c.st) c.st->join(c.s);
  GemmArgs<T> g{c.t(l.sD3), H, c.t(l.A[5]), H, (int)d.G, B, H, (int)d.Gp, Bp, 0};
  if (c.ridx) g.idx_lim = c.res_rows;
  if (c.ridx)
    launch_gemm_recon_loss<T>(g, prm + d.off[D9B], c.xbres, c.ld_xbres, with_grad, scal, c.t(l.dL), d.Gp,
                              c.f(l.losspart), c.f(l.colpart), d.Gp, c.s, c.ridx);
  else
    launch_gemm_recon_loss<T>(g, prm + d.off[D9B], (const uint32_t*)(c.ws + c.xbo), d.Gp / 32, with_grad, scal,
                              c.t(l.dL), d.Gp, c.f(l.losspart), c.f(l.colpart), d.Gp, c.s);
  int na_ok = 0, na_n = 0;
  if (norm_hdr) {  // the training call: record whether its backward takes the clip statistics
    const BigGrads<T> bg = big_grads<T>(c, Bp);
    na_ok = bg.direct ? 1 : 0;
    na_n = bg.n9 + bg.n0;
  }
  // 4) loss slot sums + the output bias's gradient (column sums of dL): nothing in the backward
  // reads them before its final join, so a training call hands the launch to the backward, which
  // puts it on the side stream behind its first fork (off the critical path, one launch and its
  // gap fewer on the caller's stream)
  const float* lpart = c.f(l.losspart);
  const int nlp = gemm_recon_grid_blocks<T>(g), nkp = Bp / kReparamRows, rt = gemm_recon_row_tiles<T>(g);
  const float *kpart = c.f(l.klpart), *cpart = c.f(l.colpart);
  const int64_t Gp = d.Gp, G = d.G;
  float* bgrad = with_grad ? grads + d.off[D9B] : nullptr;
  int* hdr = norm_hdr ? (int*)(c.ws + l.nahdr) : nullptr;
  auto tail = [=](hipStream_t s) {
    launch_fwd_tail(lpart, nlp, kpart, nkp, loss, cpart, rt, Gp, G, bgrad, hdr, na_ok, na_n, s);
  };
  // (env GM2_TAIL_MAIN: on the caller's stream, as before; A/B profiles/r03_fwd_tail_side_ab.txt)
  static const bool tail_main = std::getenv("GM2_TAIL_MAIN") != nullptr;
  if (defer_tail && !tail_main) *defer_tail = tail;
  else tail(c.s);
}

// The next training batch's gather, staged into the other input slot (gm2_batch.next)
struct NextStage {
  const gm2_batch* b = nullptr;
  int64_t xo = 0, xbo = 0;
  hipEvent_t done = nullptr;
};

// Backward. Every operand is read in the layout its producer wrote: weight gradients use MN-major P
// and Q (dW[out][in] = sum_b dY[b][out] * in[b][in]), input gradients an MN-major weight
// (dX[b][in] = sum_out dY[b][out] * W[out][in]); no transposed copy exists anywhere.
template <typename T>
void backward(const Ctx<T>& c, const gm2_batch* b, const float* prm, float* gr, const float* scal,
              const float* dmu_ext = nullptr, const float* dlv_ext = nullptr, int train = 1,
              const NextStage* nx = nullptr, std::function<void(hipStream_t)>* fwd_tail = nullptr) {
  const Dims& d = c.d;
  const Layout& l = c.lo;
  const int B = (int)b->n, Bp = (int)round_up(B, kTile);
  const int H = (int)d.H, L = (int)d.L, G = (int)d.G;
  const int Gp = (int)d.Gp, Lr = (int)d.Lr, L2r = (int)d.L2r;
  // weight gradients go to a side stream: they are off the critical path (dY -> dX -> BN -> ...)
  // and fill the tails of its launches; the join at the end orders them before the caller's work
  WsState& st = *c.st;
  const hipStream_t side = st.side_stream();
  const bool sr = side != nullptr;
  const Ctx<T> w = sr ? c.side(side) : c;
  auto fork = [&] {
    if (sr) st.order(c.s, w.s);
  };
  // The side-stream work of the first hidden layers (5, 4, 3 and the heads) would queue behind dW9
  // on the side stream anyway: it is enqueued at the fork of layer 2 instead, one ordering event in
  // place of five (each costs the main stream ~7 us; -7..-11 us per step, profiles/r03_fork_batch_ab.txt;
  // holding layer 2 as well measured +15 us). Env GM2_FORK_HOLD = the first layer whose own fork is
  // taken (6 = every layer forks), for A/Bs.
  static const int hold_from = [] {
    const char* e = std::getenv("GM2_FORK_HOLD");
    return e ? std::max(1, std::atoi(e)) : 3;
  }();
  const bool fork_batch = true;
  std::vector<std::function<void()>> held;
  auto side_work = [&](bool hold, std::function<void()> f) {
    if (hold && sr && fork_batch) {
      held.push_back(std::move(f));
      return;
    }
    f();
  };
  auto fork_flush = [&](bool hold) {
    if (hold && sr && fork_batch) return;
    fork();
    for (auto& f : held) f();
    held.clear();
  };
  // output layer: dW9[g][h] = sum_b dL[b][g] A5[b][h] ; dA5[b][h] = sum_g dL[b][g] W9[g][h]
  // (its bias gradient was summed in the forward's recon epilogue, before the fork)
  // Written as dW9^T[h][g] = sum_b A5^T[h][b] dL[b][g] with A5^T K-major (a transposed copy made
  // here) and dL MN-major, stored transposed: one transposed-read operand instead of two (the
  // 256x256 tile is LDS-read bound with two). Plans with split-K keep the both-MN-major form.
  // (Forking it last instead, beside the input-layer dWe0 GEMM, measured the same step time on one
  // GPU; first keeps gradient bucket 0 early for the data-parallel exchange.)
  const BigGrads<T> bg = big_grads<T>(c, Bp);
  double* nasq = (double*)(c.ws + l.nasq);
  // the forward's deferred tail launch (loss sums, output bias gradient): behind the first fork
  auto tail_on = [&](hipStream_t s) {
    if (fwd_tail && *fwd_tail) {
      (*fwd_tail)(s);
      *fwd_tail = nullptr;
    }
  };
  // The output-layer weight gradient (dW9, gradient bucket 0) is ordered on the side stream behind
  // an explicit point of the main stream's chain: its `dw9_at`-th kernel counted from dA5 (0 = dA5,
  // 1 = layer 5's BatchNorm backward apply, 2 = the first hidden dX GEMM, ...; env GM2_DW9_AT for
  // A/Bs). Launched alongside dA5 it would take the CUs dA5 needs; after dA5 its 860 tiles start as
  // the hidden chain's first kernels do (the chain's head start is the gap dw9_at leaves). The
  // forward tail (loss slot sums, output bias gradient, norm-ahead header) runs right in front of
  // it, on CUs dA5 no longer holds. (Rounds 3-4 had the tail in front of dW9 right after the first
  // fork: starved beside dA5 for ~360 us, it was what held dW9 back; profiles/r04_fwd_tail_after_dw9.txt.)
  // Default 2 with dW9 on its capped grid (GM2_OPT_GRID_CAP bit 1, 215 workgroups x 4 tiles): the
  // chain's BatchNorm partial and apply run before dW9 takes 215 CUs, and 41 CUs stay with the
  // chain -- 6 of 6 same-box pairs faster than 0 on the full grid (profiles/r05_dw9_cap_ab.txt).
  static const int dw9_at = [] {
    const char* e = std::getenv("GM2_DW9_AT");
    return e ? std::max(0, std::atoi(e)) : 2;
  }();
  const hipStream_t s9 = sr ? w.s : c.s;
  bool dw9_done = false;
  auto dw9_launch = [&] {
    if (dw9_done) return;
    dw9_done = true;
    const GemmArgs<T>& g9 = bg.g9;
    const bool direct9 = plan_gemm<T>(g9).splits == 1;
    fork();
    tail_on(s9);
    if (direct9) {
      // (A5^T here on the side stream; on the main stream before the fork measured ~35 us/step
      // slower, profiles/r02_a5t_placement_ab.txt)
      launch_transpose<T>(c.t(l.A[5]), H, Bp, H, c.t(l.AT5), Bp, s9);
      launch_gemm_trans<T>(g9, gr + d.off[D9W], H, s9, bg.direct ? nasq : nullptr);
    } else {
      gemm_to<T>(w, c.t(l.dL), Gp, Gp, c.t(l.A[5]), H, H, G, H, Bp, gr + d.off[D9W], nullptr, 0, H, 0, 0);
    }
    if (st.opt.grad_buckets) HIP_OK(hipEventRecord(st.bucket[0], s9));
  };
  int chain_pos = 0;
  auto chain_mark = [&] {  // after each kernel of the main stream's chain
    if (chain_pos++ == dw9_at) dw9_launch();
  };
  // dA_j = dY . W (K-major dY, MN-major W) into the slab area; when the plan allows, the GEMM's
  // epilogue also takes BatchNorm j's backward partials (sum do, sum (y-mean) do)
  bool have_part = false;
  auto dx_pre_bn = [&](const T* dY, int64_t lddy, const T* W, int64_t ldw, int K, int j) {
    GemmArgs<T> g{dY, lddy, W, ldw, B, H, K, Bp, H, 0, 1, 0};
    StoreEpi bn;
    bn.mode = 2;
    bn.part = (float2*)c.f(l.bnpart);
    bn.ldp = H;
    bn.Y = c.f(l.Y[j]);
    bn.ldy = H;
    bn.save = c.f(l.save[j]);
    bn.gamma = prm + d.off[kBlk[j][2]];
    bn.beta = prm + d.off[kBlk[j][3]];
    bn.H = H;
    have_part = launch_gemm_bn<T>(g, c.f(c.slab_off), H, nullptr, bn, c.s);
    return have_part ? 1 : gemm_to_slabs<T>(c, dY, lddy, Bp, W, ldw, H, B, H, K, H, 1, 0);
  };
  int S = dx_pre_bn(c.t(l.dL), Gp, c.t(l.sD3), H, Gp, 5);
  chain_mark();
  const int64_t shadow_w[6] = {l.sE0, l.sE1, l.sE2, l.sD0, l.sD1, l.sD2};
  for (int i = 5; i >= 0; --i) {
    const int64_t slab = (int64_t)Bp * H;
    const bool sum = S > 1;
    if (!have_part)
      launch_bn_bwd_partial(c.f(c.slab_off), S, slab, c.f(l.Y[i]), H, c.f(l.save[i]), prm + d.off[kBlk[i][2]],
                            prm + d.off[kBlk[i][3]], B, H, c.f(l.bnpart), sum ? c.f(l.DA) : nullptr, c.s);
    // bias-gradient partials go to this layer's own slice: their column sum runs on the side stream
    float* colp = c.f(l.colbwd) + (int64_t)i * l.colbwd_cap;
    const bool sync = train && st.opt.sync_bn;
    double* syncb = (double*)(c.ws + l.syncb);
    if (sync) {  // SyncBN: the batch-coupling sums of the backward over every rank's rows
      launch_bn_sync_pack(c.f(l.bnpart), B, H, 1, syncb, c.s);
      st.allreduce(syncb, 2 * H + 2, c.s);
    }
    // (input layer, bf16: its only consumer is dWe0, which reads dY0 transposed -- written that way
    // by the same pass instead of through a transpose launch)
    const bool dyt = i == 0 && sizeof(T) == 2;
    launch_bn_bwd_apply<T>(sum ? c.f(l.DA) : c.f(c.slab_off), c.f(l.Y[i]), H, c.f(l.bnpart), B, Bp, H, train,
                           c.f(l.save[i]), prm + d.off[kBlk[i][2]], prm + d.off[kBlk[i][3]], gr + d.off[kBlk[i][2]],
                           gr + d.off[kBlk[i][3]], c.t(l.dY[i]), colp, c.s, sync ? syncb : nullptr,
                           dyt ? c.t(l.dYT0) : nullptr, Bp);
    chain_mark();
    const bool hold = i >= hold_from;
    fork_flush(hold);
    side_work(hold, [&, colp, i] { launch_colsum(colp, Bp / 64, H, H, gr + d.off[kBlk[i][1]], nullptr, 0, w.s); });
    const T* dY = c.t(l.dY[i]);
    if (i == 0) {  // input layer: weight gradient only (on the main stream: nothing left to overlap)
      dw9_launch();  // (a dw9_at past the chain's end: here, beside dWe0)
      // dWe0[h][g] = sum_b dY0^T[h][b] X[b][g]: dY0^T (K-major copy) x X (MN-major)
      if (!dyt) launch_transpose<T>(dY, H, Bp, H, c.t(l.dYT0), Bp, c.s);
      // bucket 1 (every hidden-layer weight gradient) is final when the side stream's queue so far
      // is; dWe0 starts without waiting for it (the join follows the dWe0 launch: the side stream's
      // last small GEMM / column sums run beside dWe0's first tiles instead of before them)
      if (st.opt.grad_buckets) HIP_OK(hipEventRecord(st.bucket[1], w.s));
      if (input_chunked(bg, H)) {  // four row-quarter launches, bucket 2 + q final after launch q
        for (int q = 0; q < 4; ++q) {
          GemmArgs<T> gq = bg.g0;
          const int r0 = (int)input_quarter_row(d, q);
          gq.P = bg.g0.P + (int64_t)r0 * bg.g0.ldp;
          gq.M = gq.Mp = H / 4;
          if (!launch_gemm_sq<T>(gq, gr + d.off[E0W] + (int64_t)r0 * G, G, nullptr, c.s, true))
            throw Gm2Error("input-layer quarter GEMM: not a one-pass plan");
          if (st.opt.grad_buckets) HIP_OK(hipEventRecord(st.bucket[2 + q], c.s));
          st.bucket_ev[2 + q] = 2 + q;
        }
      } else {
        if (!bg.direct || !launch_gemm_sq<T>(bg.g0, gr + d.off[E0W], G, nasq + bg.n9, c.s, false))
          gemm_to<T>(c, c.t(l.dYT0), Bp, H, bg.g0.Q, bg.g0.ldq, Gp, H, G, Bp, gr + d.off[E0W], nullptr, 0, G, 1, 0,
                     bg.g0.qrow);
        // one launch: buckets 2..5 become final together, one event marks all four
        if (st.opt.grad_buckets) HIP_OK(hipEventRecord(st.bucket[2], c.s));
        for (int q = 0; q < 4; ++q) st.bucket_ev[2 + q] = 2;
      }
      if (sr) st.order(w.s, c.s);  // join: the caller's stream sees every weight gradient
      if (nx) {  // the next batch's rows -> the other input slot, on the side stream after dWe0 (beside
                 // it, it only slows the GEMM down by its own length): under the data-parallel exchange
                 // of the input-layer gradient, or beside the clip / Adam passes on one GPU
        const hipStream_t gs = sr ? w.s : c.s;
        if (sr) st.order(c.s, w.s);  // placed after dWe0 (that slot's readers, the previous step, are earlier)
        const int Bn = (int)nx->b->n;
        launch_gather_rows<T>(nx->b->data, nx->b->ld_data, nx->b->rows, Bn, G, c.t(nx->xo), Gp, Gp,
                              (int)round_up(Bn, kTile), (uint32_t*)(c.ws + nx->xbo), Gp / 32, gs);
        HIP_OK(hipEventRecord(nx->done, gs));
        // joined back before the call returns: the caller's stream orders every write this call
        // makes (workspace lifetime, device-wide syncs are not needed); the clip / Adam passes that
        // follow wait for it, which measured time-neutral (both are HBM-bound) and keeps the gather
        // beside the data-parallel exchange, which waits on bucket events instead
        if (sr) st.order(w.s, c.s);
      }
      st.recorded = st.opt.grad_buckets != 0;
      break;
    }
    if (i == 3) {  // decoder input layer, then back through the reparameterisation and the heads
      side_work(3 >= hold_from, [&, dY] { gemm_to<T>(w, dY, H, H, c.t(l.Z), Lr, Lr, H, L, Bp, gr + d.off[D0W], nullptr, 0, L, 0, 0); });
      S = gemm_to_slabs<T>(c, dY, H, Bp, c.t(l.sD0), Lr, Lr, B, L, H, L, 1, 0);
      float* colh = c.f(l.colbwd) + 6 * l.colbwd_cap;
      launch_reparam_bwd<T>(c.f(c.slab_off), S, (int64_t)Bp * L, L, c.f(l.HD), b->eps, scal, B, Bp, L, c.t(l.dH),
                            L2r, dmu_ext, dlv_ext, colh, c.s);
      fork_flush(3 >= hold_from);
      side_work(3 >= hold_from, [&, colh] {
        launch_colsum(colh, Bp / kReparamRows, 2 * L, 2 * L, gr + d.off[MUB], gr + d.off[LVB], L, w.s);
        gemm_to<T>(w, c.t(l.dH), L2r, L2r, c.t(l.A[2]), H, H, 2 * L, H, Bp, gr + d.off[MUW], gr + d.off[LVW], L, H,
                   0, 0);
      });
      S = dx_pre_bn(c.t(l.dH), L2r, c.t(l.sHD), H, (int)d.K2L, 2);
      chain_mark();
      continue;
    }
    side_work(hold, [&, dY, i] {
      gemm_to<T>(w, dY, H, H, c.t(l.A[i - 1]), H, H, H, H, Bp, gr + d.off[kBlk[i][0]], nullptr, 0, H, 0, 0);
    });
    S = dx_pre_bn(dY, H, c.t(shadow_w[i]), H, H, i - 1);
    chain_mark();
  }
}

// The sampling decode's output layer, gated per tile (extras.py:196-201, decode + threshold).
//  * bf16x3 split: activations and output weights split into bf16 (hi | lo) per 32 columns
//    (launch_split3), and the main loop (mainloop_pp, S3) sums hi.hi + hi.lo + lo.hi -- each fp32
//    product a.w up to 3.02 x 2^-16 |a| |w| (the dropped lo.lo term and the two splits' residuals),
//    i.e. per logit at most e = 4.62e-5 ||a_r||_2 ||w_g||_2 (Cauchy-Schwarz) on top of the fp32
//    accumulation the exact path has as well.
//  * Per 256 x 256 tile (genome rows x genes) the gate takes the split form when 4.62e-5 x the
//    block's largest ||a_r|| x the block's largest ||w_g|| is at most kSplitBound (1e-3); every
//    other tile runs the exact-fp32 kernel. One large activation row or weight row thus sends only
//    its own tiles to fp32. Both kernels are launched over their full grids behind the split kernels
//    and each tile's workgroup runs only on its verdict (the rest exit at once): no call waits on the
//    host. (A host read of the maxima stalled every chunk behind the previous chunk's mask copy and
//    drained the queue: 3.0 M genomes/s end to end. The first device form gated whole chunks on the
//    global maxima, so one large row or weight sent every tile to fp32.)
//  * Certified band (SURVEY.md 7 "Hard parts" (ii)): both epilogues list the elements whose logit
//    lies within coef * ||a_r|| ||w_g|| of the threshold (MaskBand) -- where the reference's own fp32
//    arithmetic, or the split, could land on either side -- and k_band_fix recomputes each listed
//    logit in fp64 from the same fp32 activations and weights and sets its mask bit from that. The
//    counts (tiles per path, band elements, bits the recompute flipped, list overflow) accumulate in
//    the workspace (DecodeCtl) for gm2_workspace_stat.
// False: not taken (the caller runs the exact path alone, without band recompute).
bool decode_split3(const Ctx<float>& c, const float* prm, int n, uint8_t* mask, int64_t ldm, uint8_t* bits,
                   int64_t ldb) {
  const Dims& d = c.d;
  const Layout& l = c.lo;
  const int H = (int)d.H, G = (int)d.G;
  const int Bq = (int)round_up(n, 2 * kTile), Gq = (int)round_up(G, 2 * kTile);
  // Preconditions of the split kernels and the two gated output-layer kernels, checked before
  // anything is launched; when one fails the caller runs the exact path alone. The output weights
  // start at off[D9W] floats into the parameter buffer, which is 2L mod 128 floats: an odd latent
  // width leaves them only 4-B aligned (launch_split3 reads 16-B pieces). The exact kernel's packed
  // stores need ldb * 8 >= its padded gene extent, the split kernel's the 256-padded one up to ldb.
  if (!l.s3a || H % 32) return false;
  if ((((uintptr_t)(prm + d.off[D9W])) | ((uintptr_t)c.f(l.A[5]))) & 15) return false;
  if (bits && ((ldb & 15) || (((uintptr_t)bits) & 15) || ldb * 8 < d.Gp)) return false;
  if (mask && !bits && (ldm < G)) return false;
  // u8 masks alone: the decode writes packed bits into the workspace and k_expand_bits writes the
  // caller's rows from them in one streaming pass (the tile epilogue's own u8 rows, at odd G never
  // 16-B aligned, cost 3.4 ms more per 65,536-genome chunk, profiles/r06_decode_u8_ab.txt)
  uint8_t* mask_out = nullptr;
  if (mask && !bits) {
    if (!l.s3bits || l.s3ldb * 8 < d.Gp) return false;
    mask_out = mask;
    mask = nullptr;
    bits = (uint8_t*)(c.ws + l.s3bits);
    ldb = l.s3ldb;
  }
  unsigned* ctl = (unsigned*)(c.ws + l.s3ctl);
  unsigned* ablk = ctl + DecodeCtl::kBlk;
  unsigned* wblk = ablk + Bq / 256;
  bf16_t* a3 = (bf16_t*)(c.ws + l.s3a);
  bf16_t* w3 = (bf16_t*)(c.ws + l.s3w);
  float* rn = c.f(l.s3rn);
  float* cn = c.f(l.s3cn);
  uint2* list = (uint2*)(c.ws + l.s3band);
  const float* w9 = prm + d.off[D9W];
  HIP_OK(hipMemsetAsync(ctl + DecodeCtl::kTilesSplit, 0, (DecodeCtl::kBlk - DecodeCtl::kTilesSplit + Bq / 256 + Gq / 256) * 4,
                        c.s));
  const bool single = opts().sample_single != 0 && H % 64 == 0;  // (the single GEMM's K = H: 64-wide K-tiles)
  bf16_t* a1 = (bf16_t*)(c.ws + l.s3a1);
  bf16_t* w1 = (bf16_t*)(c.ws + l.s3w1);
  launch_split3(c.f(l.A[5]), H, n, Bq, H, a3, 2 * H, rn, ablk, c.s, single ? a1 : nullptr);
  launch_split3(w9, H, G, Gq, H, w3, 2 * H, cn, wblk, c.s, single ? w1 : nullptr);
  if (c.st) {
    c.st->decode_cum = (const unsigned long long*)(ctl + DecodeCtl::kCum);
    c.st->decode_ovf = (const unsigned long long*)(c.ws + l.s3ovf);
  }
  // band half-widths per unit ||a_r|| ||w_g|| (MaskBand): single tiles carry the operands' bf16
  // rounding and the fp32 accumulation of their H products, split tiles the split's own error and the
  // fp32 accumulation of its 3H products, exact tiles the fp32 accumulation of H products; all, the
  // reference's own fp32 accumulation of H products
  const double gH = band_gamma((double)H), g3H = band_gamma(3.0 * H);
  // (the split and single kernels' tiles keep their band elements in their own slots -- the tile
  // grid is the same and each tile runs in one of them; the exact kernel's, rare, go to the shards)
  const int tiles = (Bq / 256) * (Gq / 256);
  MaskBand bs{rn, cn, (float)(kSplitUnit * 1.01 + g3H + gH), ctl + DecodeCtl::kCounts, list, kBandShardCap};
  MaskBand be = bs;
  be.coef = (float)(2.0 * gH);
  bs.tlist = (uint2*)(c.ws + l.s3tlist);
  bs.tcount = (unsigned*)(c.ws + l.s3tcount);
  bs.tfound = ctl + DecodeCtl::kTileFound;
  bs.tslots = kBandTileSlots;
  MaskBand b1 = bs;
  b1.coef = (float)(kSingleUnit * 1.01 + 2.0 * gH);
  b1.drop_overflow = 1;
  b1.tiles_done = ctl + DecodeCtl::kTilesSingle;
  HIP_OK(hipMemsetAsync(bs.tcount, 0, (size_t)tiles * 4, c.s));
  // band-list overflow: entries past a shard's capacity flag their 256 x 256 block, which
  // k_band_tile_fix then recomputes whole in fp64 (no bit is left as a bf16 tier decided it)
  unsigned* ovf = (unsigned*)(c.ws + l.s3ovf);
  HIP_OK(hipMemsetAsync(ovf + Layout::kOvfCount, 0, (size_t)(Layout::kOvfFlags - Layout::kOvfCount + tiles) * 4, c.s));
  bs.cap = (unsigned)std::min<int>(opts().band_cap, (int)kBandShardCap);
  bs.oflag = ovf + Layout::kOvfFlags;
  bs.olist = bs.oflag + tiles;
  bs.ocount = ovf + Layout::kOvfCount;
  bs.obn = Gq / 256;
  bs.oblocks = (unsigned)tiles;
  be.cap = bs.cap;
  be.oflag = bs.oflag;
  be.olist = bs.olist;
  be.ocount = bs.ocount;
  be.obn = bs.obn;
  be.oblocks = bs.oblocks;
  const int on = single ? 1 : 0;
  const double single_bound = opts().single_bound_milli * 1e-3;  // (GM2_OPT_SAMPLE_SINGLE_BOUND, for A/Bs and tests)
  GemmArgs<bf16_t> g{a3, 2 * H, w3, 2 * H, n, G, 2 * H, Bq, Gq, 0};
  const MaskGate gs{ablk, wblk, 1, ctl + DecodeCtl::kTilesSplit, on, single_bound};
  if (single) {  // both bf16 tiers in one launch (a single tile whose band overflows re-runs as split)
    GemmArgs<bf16_t> g1{a1, H, w1, H, n, G, H, Bq, Gq, 0};
    launch_gemm_mask_tiered(g1, g, prm + d.off[D9B], mask, ldm, bits, ldb, c.s,
                            MaskGate{ablk, wblk, 3, ctl + DecodeCtl::kTilesSingle, on, single_bound}, b1, gs, bs);
  } else {
    launch_gemm_mask<bf16_t>(g, prm + d.off[D9B], mask, ldm, nullptr, 0, c.s, bits, ldb, nullptr, nullptr, 0, 0.5f,
                             true, gs, bs);
  }
  GemmArgs<float> ge{c.f(l.A[5]), H, c.f(l.sD3), H, n, G, H, (int)round_up(n, kTile), (int)d.Gp, 0};
  launch_gemm_mask<float>(ge, prm + d.off[D9B], mask, ldm, nullptr, 0, c.s, bits, ldb, nullptr, nullptr, 0, 0.5f,
                          false, MaskGate{ablk, wblk, 2, ctl + DecodeCtl::kTilesExact, on, single_bound}, be);
  launch_band_fix(bs, tiles, c.f(l.A[5]), H, w9, H, prm + d.off[D9B], H, bits, ldb, mask, ldm,
                  ctl + DecodeCtl::kFlips, c.s);
  launch_band_tile_fix(bs, c.f(l.A[5]), H, w9, H, prm + d.off[D9B], H, n, G, bits, ldb, mask, ldm,
                       ctl + DecodeCtl::kFlips, c.s);
  launch_decode_stats(ctl + DecodeCtl::kTilesSplit, ctl + DecodeCtl::kTilesExact, ctl + DecodeCtl::kTilesSingle,
                      ctl + DecodeCtl::kCounts, ctl + DecodeCtl::kTileFound, ctl + DecodeCtl::kFlips, bs.cap,
                      (unsigned long long*)(ctl + DecodeCtl::kCum), bs.ocount, (unsigned long long*)ovf, c.s);
  if (mask_out) launch_expand_bits(bits, ldb, n, G, mask_out, ldm, c.s);
  return true;
}

template <typename T>
void decode_chain(const Ctx<T>& c, const float* prm, float* bn, int n, uint8_t* mask, int64_t ldm, float* probs,
                  int64_t ldpr, uint8_t* bits = nullptr, int64_t ldb = 0) {
  const Dims& d = c.d;
  const Layout& l = c.lo;
  const int Bp = (int)round_up(n, kTile), H = (int)d.H;
  const T* in = c.t(l.Z);
  int64_t ldin = d.Lr;
  int Kin = (int)d.Lp;
  int64_t ldw = d.Lr;
  const int64_t shadow_in[3] = {l.sD0, l.sD1, l.sD2};
  for (int j = 0; j < 3; ++j) {
    const int i = 3 + j;
    linear_pre_bn<T>(c, in, ldin, Bp, c.t(shadow_in[j]), ldw, n, H, Kin, prm + d.off[kBlk[i][1]], c.f(l.Y[i]),
                     c.f(l.bnpart), false);
    launch_bn_fwd_apply<T>(c.f(l.Y[i]), H, c.f(l.bnpart), n, Bp, H, 0, prm + d.off[kBlk[i][2]], prm + d.off[kBlk[i][3]],
                           bn + (int64_t)i * 2 * H, bn + (int64_t)i * 2 * H + H, nullptr, c.t(l.A[i]), c.s);
    in = c.t(l.A[i]);
    ldin = H;
    Kin = H;
    ldw = H;
  }
  if constexpr (std::is_same_v<T, float>) {
    if (!probs && opts().sample_split && decode_split3(c, prm, n, mask, ldm, bits, ldb)) return;
  }
  if (c.st) c.st->exact_decodes++;
  GemmArgs<T> g{c.t(l.A[5]), H, c.t(l.sD3), H, n, (int)d.G, H, Bp, (int)d.Gp, 0};
  launch_gemm_mask<T>(g, prm + d.off[D9B], mask, ldm, probs, ldpr, c.s, bits, ldb);
}

// make `s` wait for a pending stage on `ws` and forget it (the caller is about to write slot 0)
void drop_stage(WsState& st, hipStream_t s) {
  if (st.slot.staged) HIP_OK(hipStreamWaitEvent(s, st.slot_done, 0));
  st.slot.staged = false;
}

// SyncBN, a rank with no rows in this global batch: zero gradient and loss sums, the 12 all-reduces
// with zero contributions in the order the ranks with rows issue them, and the same running-statistics
// update (the global batch's); bucket events recorded so a gradient exchange can follow
void sync_bn_no_rows(const Layout& lo, float* gr, float* bn, double* loss, void* ws, hipStream_t s, WsState& st) {
  const Dims& d = lo.d;
  const int64_t H = d.H, n = 2 * H + 2;
  double* syncb = (double*)((char*)ws + lo.syncb);
  HIP_OK(hipMemsetAsync(gr, 0, (size_t)d.off[NP] * 4, s));
  HIP_OK(hipMemsetAsync(loss, 0, 3 * sizeof(double), s));
  for (int i = 0; i < 6; ++i) {
    HIP_OK(hipMemsetAsync(syncb, 0, (size_t)n * 8, s));
    st.allreduce(syncb, n, s);
    launch_bn_sync_running(syncb, (int)H, bn + (int64_t)i * 2 * H, bn + (int64_t)i * 2 * H + H, s);
  }
  for (int i = 5; i >= 0; --i) {
    HIP_OK(hipMemsetAsync(syncb, 0, (size_t)n * 8, s));
    st.allreduce(syncb, n, s);
  }
  if (st.opt.grad_buckets)
    for (int b = 0; b < GM2_GRAD_BUCKETS; ++b) {
      HIP_OK(hipEventRecord(st.bucket[b], s));
      st.bucket_ev[b] = b;
    }
  st.recorded = st.opt.grad_buckets != 0;
}

// gm2_batch.resident usable in place for this training call: its precision, padding and alignment,
// and GEMM plans that take zero-copy rows (bf16 256x256 ping-pong); otherwise the rows are gathered
template <typename T>
bool zero_copy_ok(const Ctx<T>& c, const gm2_batch* b) {
  const Dims& d = c.d;
  if (!b->resident || b->resident_prec != c.lo.prec || sizeof(T) != 2) return false;
  if (!b->resident_bits || b->resident_rows < 0 || b->resident_rows > INT32_MAX - 1) return false;
  if (b->ld_resident < d.Gp || b->ld_resident % 64 || ((uintptr_t)b->resident & 15)) return false;
  if (b->ld_resident_bits < d.Gp / 32 || b->ld_resident_bits % 4 || ((uintptr_t)b->resident_bits & 15)) return false;
  const int B = (int)b->n, Bp = (int)round_up(B, kTile), H = (int)d.H;
  if (B < 1 || Bp % (2 * kTile)) return false;
  GemmArgs<T> enc{(const T*)b->resident, b->ld_resident, c.t(c.lo.sE0), d.Gp, B, H, (int)d.Gp, Bp, H, 0};
  enc.prow = (const int32_t*)1;
  GemmArgs<T> dwe0{c.t(c.lo.dYT0), Bp, (const T*)b->resident, b->ld_resident, H, (int)d.G, Bp, H, (int)d.Gp, 0, 1, 0};
  dwe0.qrow = (const int32_t*)1;
  return gemm_idx_ok<T>(enc) && gemm_idx_ok<T>(dwe0);
}

template <typename T>
void run_train(const Layout& lo, const gm2_batch* b, const float* prm, float* gr, float* bn, const float* scal,
               double* loss, void* ws, void* strm, WsState& st) {
  if (b->n == 0 && st.opt.sync_bn) {
    st.join((hipStream_t)strm);  // (it zeroes the whole gradient buffer)
    if (st.slot.staged) HIP_OK(hipStreamWaitEvent((hipStream_t)strm, st.slot_done, 0));
    st.slot.staged = false;
    sync_bn_no_rows(lo, gr, bn, loss, ws, (hipStream_t)strm, st);
    return;
  }
  Ctx<T> c(lo, ws, strm, &st);
  if (zero_copy_ok<T>(c, b)) {  // the resident matrix's rows in place: no gather, no staging
    c.ridx = (const int32_t*)((char*)ws + lo.ridx);
    c.xres = (const T*)b->resident;
    c.ld_xres = b->ld_resident;
    c.xbres = b->resident_bits;
    c.ld_xbres = b->ld_resident_bits;
    c.res_rows = b->resident_rows + 1;
    drop_stage(st, c.s);
    std::function<void(hipStream_t)> tail;
    forward<T>(c, b, prm, bn, 1, 1, scal, loss, gr, nullptr, 0, nullptr, 0.5f, true, false, &tail);
    backward<T>(c, b, prm, gr, scal, nullptr, nullptr, 1, nullptr, &tail);
    return;
  }
  SlotState& ss = st.slot;
  const bool hit = ss.staged && ss.prec == lo.prec && ss.total == lo.total && ss.data == b->data &&
                   ss.ld == b->ld_data && ss.rows == b->rows && ss.n == b->n;
  if (ss.staged) HIP_OK(hipStreamWaitEvent(c.s, st.slot_done, 0));
  const int slot = hit ? ss.slot : 0;
  c.xo = slot ? lo.X1 : lo.X;
  c.xbo = slot ? lo.XB1 : lo.XB;
  ss.staged = false;
  NextStage nx;
  const gm2_batch* nb = b->next;
  if (nb) {
    if (nb->n <= 0 || nb->n > lo.d.Bm) throw Gm2Error("next batch: rows %lld outside (0, batch_max]", (long long)nb->n);
    check_batch_data(nb, lo.d, "next batch");
    nx.b = nb;
    nx.xo = slot ? lo.X : lo.X1;
    nx.xbo = slot ? lo.XB : lo.XB1;
    nx.done = st.slot_done;
  }
  std::function<void(hipStream_t)> tail;
  forward<T>(c, b, prm, bn, 1, 1, scal, loss, gr, nullptr, 0, nullptr, 0.5f, true, hit, &tail);
  backward<T>(c, b, prm, gr, scal, nullptr, nullptr, 1, nb ? &nx : nullptr, &tail);
  if (nb) {
    ss.staged = true;
    ss.slot = slot ^ 1;
    ss.data = nb->data;
    ss.ld = nb->ld_data;
    ss.rows = nb->rows;
    ss.n = nb->n;
    ss.prec = lo.prec;
    ss.total = lo.total;
  }
}

// guarded body of a C-ABI call on workspace `ws`: its state, with its options in scope
template <typename F>
int with_ws(void* ws, F&& f) {
  return guarded([&] {
    WsState& st = ws_state(ws);
    OptionScope scope(st.opt);
    f(st);
  });
}

// the same for a call that reads or writes parameters, moments or GEMM shadows from its first
// launch on: it first joins a deferred output-layer Adam update (the training call instead waits
// right before the output layer, so the update overlaps its first half)
template <typename F>
int with_ws_joined(void* ws, void* stream, F&& f) {
  return with_ws(ws, [&](WsState& st) {
    st.join((hipStream_t)stream);
    f(st);
  });
}

}  // namespace

// =================================================================================================
extern "C" {

const char* gm2_last_error(void) { return g_err.c_str(); }
int gm2_abi_version(void) { return GM2_ABI_VERSION; }

int gm2_param_count(const gm2_dims* d, int64_t* n) {
  return guarded([&] { *n = make_dims(d).off[NP]; });
}

int gm2_param_offsets(const gm2_dims* d, int64_t* off) {
  return guarded([&] {
    const Dims x = make_dims(d);
    for (int i = 0; i <= NP; ++i) off[i] = x.off[i];
  });
}

int gm2_workspace_size(const gm2_dims* d, int prec, size_t* bytes) {
  return guarded([&] { *bytes = (size_t)make_layout(d, prec).total; });
}

int gm2_workspace_init(const gm2_dims* d, int prec, void* ws, size_t ws_bytes, void* stream) {
  return guarded([&] {
    const Layout lo = make_layout(d, prec);
    if ((size_t)lo.total > ws_bytes) throw Gm2Error("workspace too small: %zu < %lld", ws_bytes, (long long)lo.total);
    if ((uintptr_t)ws & 255) throw Gm2Error("workspace must be 256-B aligned");
    ws_reset(ws);  // a new (or reused) workspace: process-default options, no staged batch
    HIP_OK(hipMemsetAsync(ws, 0, (size_t)lo.total, (hipStream_t)stream));
  });
}

int gm2_sync_shadows(const gm2_dims* d, int prec, const float* params, void* ws, void* stream) {
  return with_ws_joined(ws, stream, [&](WsState& st) {
    const Layout lo = make_layout(d, prec);
    if (prec == GM2_F32) {
      Ctx<float> c(lo, ws, stream, &st);
      launch_shadow_sync<float>(make_table(c), params, c.s);
    } else {
      Ctx<bf16_t> c(lo, ws, stream, &st);
      launch_shadow_sync<bf16_t>(make_table(c), params, c.s);
    }
  });
}

int gm2_resident_layout(int64_t S, int64_t G, int prec, int64_t* ld, int64_t* ld_bits, int64_t* rows_alloc,
                        size_t* bytes, size_t* bits_bytes) {
  return guarded([&] {
    if (S < 0 || S > INT32_MAX - 64 || G <= 0 || (prec != GM2_F32 && prec != GM2_BF16))
      throw Gm2Error("resident layout: S=%lld G=%lld prec=%d", (long long)S, (long long)G, prec);
    const int64_t l = round_up(G, 2 * kTile), r = round_up(S + 1, 64);
    *ld = l;
    *ld_bits = l / 32;
    *rows_alloc = r;
    *bytes = (size_t)(r * l * (prec == GM2_F32 ? 4 : 2));
    *bits_bytes = (size_t)(r * (l / 32) * 4);
  });
}

int gm2_resident_build(const uint8_t* data, int64_t ld_data, int64_t S, int64_t G, int prec, void* out,
                       uint32_t* bits, void* stream) {
  return guarded([&] {
    int64_t l = 0, lb = 0, r = 0;
    size_t by = 0, bb = 0;
    if (gm2_resident_layout(S, G, prec, &l, &lb, &r, &by, &bb) != 0) throw Gm2Error("%s", g_err.c_str());
    if (!out || !bits || ((uintptr_t)out & 15) || ((uintptr_t)bits & 15)) throw Gm2Error("resident: null or misaligned output");
    if (S > 0 && (!data || ld_data % 16 || ld_data < G || ((uintptr_t)data & 15)))
      throw Gm2Error("resident: data rows must be 16-B aligned with ld_data (%lld) a multiple of 16 and >= G",
                     (long long)ld_data);
    // the gather with identity rows: rows < S copied (0/1 -> T, target bits), rows S.. r-1 and
    // columns G.. ld-1 zero
    const uint8_t* src = S > 0 ? data : (const uint8_t*)out;
    const int64_t lds = S > 0 ? ld_data : 16;
    if (prec == GM2_F32)
      launch_gather_rows<float>(src, lds, nullptr, (int)S, (int)G, (float*)out, l, (int)l, (int)r, bits, lb,
                                (hipStream_t)stream);
    else
      launch_gather_rows<bf16_t>(src, lds, nullptr, (int)S, (int)G, (bf16_t*)out, l, (int)l, (int)r, bits, lb,
                                 (hipStream_t)stream);
  });
}

int gm2_train_fwd_bwd(const gm2_dims* d, int prec, const gm2_batch* batch, const float* params, float* grads,
                      float* bn_running, const float* scalars, double* loss, void* ws, void* stream) {
  return with_ws(ws, [&](WsState& st) {
    const Layout lo = make_layout(d, prec);
    if (prec == GM2_F32) run_train<float>(lo, batch, params, grads, bn_running, scalars, loss, ws, stream, st);
    else run_train<bf16_t>(lo, batch, params, grads, bn_running, scalars, loss, ws, stream, st);
  });
}

int gm2_grad_norm(const gm2_dims* d, int prec, const float* params, const float* grads, const float* scalars,
                  double* loss, void* ws, void* stream) {
  return with_ws_joined(ws, stream, [&](WsState& st) {
    const Layout lo = make_layout(d, prec);
    const int64_t n = lo.d.off[NP];
    const int nb = grad_stats_blocks(n);
    double* part = (double*)((char*)ws + lo.gradpart);
    float* clip = (float*)((char*)ws + lo.clip);
    NormAhead na;
    na.hdr = (const int*)((char*)ws + lo.nahdr);
    na.sq = (const double*)((char*)ws + lo.nasq);
    na.lo0 = lo.d.off[E0W], na.hi0 = lo.d.off[E0B], na.lo9 = lo.d.off[D9W], na.hi9 = lo.d.off[D9B];
    launch_grad_stats(params, grads, n, scalars, part, nb, na, (hipStream_t)stream);
    launch_grad_finalize(part, nb, scalars, clip, loss + 3, na, (hipStream_t)stream);  // loss[3], loss[4]
  });
}

int gm2_adam_step(const gm2_dims* d, int prec, float* params, const float* grads, float* m, float* v,
                  const float* scalars, void* ws, void* stream) {
  return with_ws_joined(ws, stream, [&](WsState& st) {
    const Layout lo = make_layout(d, prec);
    const float* clip = (const float*)((char*)ws + lo.clip);
    auto run = [&](auto tag) {
      using T = decltype(tag);
      Ctx<T> c(lo, ws, stream, &st);
      const TensorTable all = make_table(c, 1);
      if (!st.opt.defer_adam || !st.opt.side_stream) {
        launch_adam_fused<T>(all, grads, params, m, v, scalars, clip, c.s);
        return;
      }
      // every tensor but the output layer now; decoder.9.{weight,bias} (the table's last two
      // entries, half the bytes at v0) queued with a copy of the scalar block (see WsState::kick)
      float* qs = (float*)((char*)ws + lo.adamscal);
      launch_adam_fused<T>(table_range(all, 0, all.n - 2), grads, params, m, v, scalars, clip, c.s, 0, qs);
      WsState::QueuedAdam& q = st.qadam;
      q.queued = true;
      q.prec = prec;
      q.tt = table_range(all, all.n - 2, all.n);
      q.g = grads;
      q.p = params;
      q.m = m;
      q.v = v;
      q.scal = qs;
      q.clip = clip;
    };
    if (prec == GM2_F32) run(float{});
    else run(bf16_t{});
  });
}

int gm2_eval_forward(const gm2_dims* d, int prec, const gm2_batch* batch, const float* params,
                     const float* bn_running, const float* scalars, double* loss, void* ws, void* stream) {
  return with_ws_joined(ws, stream, [&](WsState& st) {
    const Layout lo = make_layout(d, prec);
    drop_stage(st, (hipStream_t)stream);  // these write input slot 0
    float* bn = const_cast<float*>(bn_running);  // eval mode never writes running stats
    if (prec == GM2_F32) {
      Ctx<float> c(lo, ws, stream, &st);
      forward<float>(c, batch, params, bn, 0, 0, scalars, loss, nullptr);
    } else {
      Ctx<bf16_t> c(lo, ws, stream, &st);
      forward<bf16_t>(c, batch, params, bn, 0, 0, scalars, loss, nullptr);
    }
  });
}

int gm2_decode_mask(const gm2_dims* d, const float* params, const float* bn_running, const float* z, int64_t n,
                    uint8_t* mask, int64_t ld_mask, float* probs, int64_t ld_probs, void* ws, void* stream) {
  return with_ws_joined(ws, stream, [&](WsState& st) {
    const Layout lo = make_layout(d, GM2_F32);
    if (n <= 0 || n > lo.d.Bm) throw Gm2Error("decode rows %lld outside (0, batch_max]", (long long)n);
    if (ld_mask < lo.d.G || (probs && ld_probs < lo.d.G)) throw Gm2Error("decode: ld < G");
    Ctx<float> c(lo, ws, stream, &st);
    // z [n][L] -> Z [Bm][Lp] (pad columns stay zero from workspace init)
    HIP_OK(hipMemcpy2DAsync(c.f(lo.Z), lo.d.Lr * 4, z, lo.d.L * 4, lo.d.L * 4, n, hipMemcpyDeviceToDevice, c.s));
    decode_chain<float>(c, params, const_cast<float*>(bn_running), (int)n, mask, ld_mask, probs, ld_probs);
  });
}

int64_t gm2_packed_row_bytes(int64_t G) { return round_up(G, kTile) / 8; }

int gm2_mask_count_groups(const uint8_t* bits, int64_t n, int64_t ld_bits, const int32_t* group_offsets,
                          int64_t n_groups, const int32_t* positions, int32_t* counts, void* stream) {
  return guarded([&] {
    if (n < 0 || n_groups < 0 || (n && (!bits || !counts)) || (n_groups && (!group_offsets || !positions)))
      throw Gm2Error("mask_count_groups: bad arguments");
    if (n_groups == 0) {
      HIP_OK(hipMemsetAsync(counts, 0, (size_t)n * 4, (hipStream_t)stream));
      return;
    }
    launch_count_groups(bits, n, ld_bits, group_offsets, n_groups, positions, counts, (hipStream_t)stream);
  });
}

int gm2_mask_row_offsets(const uint8_t* bits, int64_t n, int64_t ld_bits, const uint8_t* keep_bits, int64_t* offsets,
                         void* stream) {
  return guarded([&] {
    if (n < 0 || !offsets || (n && !bits) || (ld_bits & 15)) throw Gm2Error("mask_row_offsets: bad arguments");
    launch_row_offsets(bits, n, ld_bits, keep_bits, offsets, (hipStream_t)stream);
  });
}

int gm2_mask_compact(const uint8_t* bits, int64_t n, int64_t ld_bits, const uint8_t* keep_bits, const int64_t* offsets,
                     int32_t* indices, void* stream) {
  return guarded([&] {
    if (n < 0 || (n && (!bits || !offsets)) || (ld_bits & 15)) throw Gm2Error("mask_compact: bad arguments");
    launch_compact(bits, n, ld_bits, keep_bits, offsets, indices, (hipStream_t)stream);
  });
}

int gm2_decode_bits(const gm2_dims* d, const float* params, const float* bn_running, const float* z, int64_t n,
                    uint8_t* bits, int64_t ld_bits, float* probs, int64_t ld_probs, void* ws, void* stream) {
  return with_ws_joined(ws, stream, [&](WsState& st) {
    const Layout lo = make_layout(d, GM2_F32);
    if (n <= 0 || n > lo.d.Bm) throw Gm2Error("decode rows %lld outside (0, batch_max]", (long long)n);
    if (ld_bits < gm2_packed_row_bytes(lo.d.G) || (probs && ld_probs < lo.d.G)) throw Gm2Error("decode_bits: ld too small");
    Ctx<float> c(lo, ws, stream, &st);
    HIP_OK(hipMemcpy2DAsync(c.f(lo.Z), lo.d.Lr * 4, z, lo.d.L * 4, lo.d.L * 4, n, hipMemcpyDeviceToDevice, c.s));
    decode_chain<float>(c, params, const_cast<float*>(bn_running), (int)n, nullptr, 0, probs, ld_probs, bits, ld_bits);
  });
}

int gm2_recon_counts(const gm2_dims* d, int prec, const gm2_batch* batch, const float* params, const float* bn_running,
                     float threshold, int32_t* counts, void* ws, void* stream) {
  return with_ws_joined(ws, stream, [&](WsState& st) {
    const Layout lo = make_layout(d, prec);
    drop_stage(st, (hipStream_t)stream);  // these write input slot 0
    if (!batch->eps) throw Gm2Error("recon_counts: eps required (model(x) samples z)");
    if (!counts) throw Gm2Error("recon_counts: counts required");
    HIP_OK(hipMemsetAsync(counts, 0, (size_t)batch->n * 3 * 4, (hipStream_t)stream));
    float* bn = const_cast<float*>(bn_running);  // eval mode never writes running stats
    auto run = [&](auto tag) {
      using T = decltype(tag);
      Ctx<T> c(lo, ws, stream, &st);
      forward<T>(c, batch, params, bn, 0, 0, nullptr, nullptr, nullptr, nullptr, 0, counts, threshold);
    };
    if (prec == GM2_F32) run(float{});
    else run(bf16_t{});
  });
}

int gm2_encode(const gm2_dims* d, int prec, const gm2_batch* batch, const float* params, const float* bn_running,
               float* mu, float* logvar, void* ws, void* stream) {
  return with_ws_joined(ws, stream, [&](WsState& st) {
    const Layout lo = make_layout(d, prec);
    drop_stage(st, (hipStream_t)stream);  // these write input slot 0
    gm2_batch b = *batch;
    auto run = [&](auto tag) {
      using T = decltype(tag);
      Ctx<T> c(lo, ws, stream, &st);
      const Dims& dd = c.d;
      const int B = (int)b.n, Bp = (int)round_up(B, kTile), H = (int)dd.H, L = (int)dd.L;
      if (B <= 0 || B > dd.Bm) throw Gm2Error("encode rows outside (0, batch_max]");
      check_batch_data(&b, dd, "encode");
      float* bn = const_cast<float*>(bn_running);
      launch_gather_rows<T>(b.data, b.ld_data, b.rows, B, (int)dd.G, c.t(lo.X), dd.Gp, (int)dd.Gp, Bp, nullptr, 0,
                            c.s);
      const T* in = c.t(lo.X);
      int64_t ldin = dd.Gp;
      int Kin = (int)dd.Gp;
      const int64_t sh[3] = {lo.sE0, lo.sE1, lo.sE2};
      for (int i = 0; i < 3; ++i) {
        linear_pre_bn<T>(c, in, ldin, Bp, c.t(sh[i]), Kin, B, H, Kin, params + dd.off[kBlk[i][1]], c.f(lo.Y[i]),
                         c.f(lo.bnpart), false);
        launch_bn_fwd_apply<T>(c.f(lo.Y[i]), H, c.f(lo.bnpart), B, Bp, H, 0, params + dd.off[kBlk[i][2]],
                               params + dd.off[kBlk[i][3]], bn + (int64_t)i * 2 * H, bn + (int64_t)i * 2 * H + H,
                               nullptr, c.t(lo.A[i]), c.s);
        in = c.t(lo.A[i]);
        ldin = H;
        Kin = H;
      }
      const int S = gemm_to_slabs<T>(c, c.t(lo.A[2]), H, Bp, c.t(lo.sHD), H, (int)dd.L2r, B, 2 * L, H, 2 * L);
      launch_reparam<T>(c.f(lo.slabs), S, (int64_t)Bp * 2 * L, L, params + dd.off[MUB], params + dd.off[LVB], nullptr,
                        B, Bp, c.f(lo.HD), c.t(lo.Z), dd.Lr, nullptr, 0, 0, c.f(lo.klpart), c.s);
      if (mu) HIP_OK(hipMemcpy2DAsync(mu, L * 4, c.f(lo.HD), 2 * L * 4, L * 4, B, hipMemcpyDeviceToDevice, c.s));
      if (logvar)
        HIP_OK(hipMemcpy2DAsync(logvar, L * 4, c.f(lo.HD) + L, 2 * L * 4, L * 4, B, hipMemcpyDeviceToDevice, c.s));
    };
    if (prec == GM2_F32) run(float{});
    else run(bf16_t{});
  });
}

int gm2_gemm(int prec, int pk, int qk, const void* P, int64_t ldp, const void* Q, int64_t ldq, float* C, int64_t ldc,
             int64_t M, int64_t N, int64_t K, int splits, float* slab_ws, void* stream) {
  return guarded([&] {
    auto run = [&](auto tag) {
      using T = decltype(tag);
      GemmArgs<T> g{(const T*)P, ldp, (const T*)Q, ldq, (int)M, (int)N, (int)K, (int)round_up(M, kTile),
                    (int)round_up(N, kTile), 0, pk ? 1 : 0, qk ? 1 : 0};
      if (splits < 0) splits = plan_gemm(g).splits;  // the hot path's own tile / split-K plan
      if (splits == 0 || splits == 1) {
        launch_gemm_store<T>(g, 1, C, nullptr, 0, ldc, 0, nullptr, (hipStream_t)stream);
      } else {
        if (!slab_ws) throw Gm2Error("gemm: split-K needs slab_ws");
        const int S = launch_gemm_store<T>(g, splits, slab_ws, nullptr, 0, ldc, (int64_t)M * ldc, nullptr,
                                           (hipStream_t)stream);
        // sum the slabs column-block-wise: treat [S][M*ldc] as rows
        launch_colsum(slab_ws, S, M * ldc, M * ldc, C, nullptr, 0, (hipStream_t)stream);
      }
    };
    if (prec == GM2_F32) run(float{});
    else if (prec == GM2_BF16) run(bf16_t{});
    else throw Gm2Error("bad precision");
  });
}

int gm2_forward(const gm2_dims* d, int prec, const gm2_batch* batch, const float* params, float* bn_running,
                int train, float* probs, int64_t ld_probs, float* mu, float* logvar, void* ws, void* stream) {
  return with_ws_joined(ws, stream, [&](WsState& st) {
    const Layout lo = make_layout(d, prec);
    drop_stage(st, (hipStream_t)stream);  // these write input slot 0
    if (!probs || ld_probs < lo.d.G) throw Gm2Error("forward: probs required, ld_probs >= G");
    if (!batch->eps) throw Gm2Error("forward: eps required (model.py:102 draws it)");
    auto run = [&](auto tag) {
      using T = decltype(tag);
      Ctx<T> c(lo, ws, stream, &st);
      forward<T>(c, batch, params, bn_running, train, 0, nullptr, nullptr, nullptr, probs, ld_probs);
      const int64_t L = lo.d.L, B = batch->n;
      if (mu) HIP_OK(hipMemcpy2DAsync(mu, L * 4, c.f(lo.HD), 2 * L * 4, L * 4, B, hipMemcpyDeviceToDevice, c.s));
      if (logvar)
        HIP_OK(hipMemcpy2DAsync(logvar, L * 4, c.f(lo.HD) + L, 2 * L * 4, L * 4, B, hipMemcpyDeviceToDevice, c.s));
    };
    if (prec == GM2_F32) run(float{});
    else run(bf16_t{});
  });
}

int gm2_backward_outputs(const gm2_dims* d, int prec, const gm2_batch* batch, const float* params, int train,
                         const float* probs, int64_t ld_probs, const float* dprobs, const float* dmu,
                         const float* dlogvar, float* grads, void* ws, void* stream) {
  return with_ws_joined(ws, stream, [&](WsState& st) {
    const Layout lo = make_layout(d, prec);
    drop_stage(st, (hipStream_t)stream);  // these write input slot 0
    if (!probs || !dprobs || ld_probs < lo.d.G) throw Gm2Error("backward_outputs: probs / dprobs required");
    auto run = [&](auto tag) {
      using T = decltype(tag);
      Ctx<T> c(lo, ws, stream, &st);
      const Dims& dd = c.d;
      const int B = (int)batch->n, Bp = (int)round_up(B, kTile);
      if (B <= 0 || B > dd.Bm) throw Gm2Error("backward_outputs: rows outside (0, batch_max]");
      launch_sigmoid_bwd<T>(probs, dprobs, ld_probs, B, Bp, (int)dd.G, (int)dd.Gp, c.t(lo.dL), dd.Gp, c.f(lo.colpart),
                            c.s);
      launch_colsum(c.f(lo.colpart), Bp / 64, dd.Gp, dd.G, grads + dd.off[D9B], nullptr, 0, c.s);
      // the fused loss terms are absent here: beta = 0 in a private scalar block
      float* scal0 = c.f(lo.scal0);
      HIP_OK(hipMemsetAsync(scal0, 0, GM2_NUM_SCALARS * 4, c.s));
      backward<T>(c, batch, params, grads, scal0, dmu, dlogvar, train);
    };
    if (prec == GM2_F32) run(float{});
    else run(bf16_t{});
  });
}

int gm2_reparameterize(int64_t n, const float* mu, const float* logvar, const float* eps, float* z,
                       const float* dz, float* dmu, float* dlogvar, void* stream) {
  return guarded([&] {
    if (!mu || !logvar || !eps || (!z && !dz) || (dz && (!dmu || !dlogvar)))
      throw Gm2Error("reparameterize: bad pointers");
    if (n < 0) throw Gm2Error("reparameterize: negative n %lld", (long long)n);
    launch_reparameterize(n, mu, logvar, eps, z, dz, dmu, dlogvar, (hipStream_t)stream);
  });
}

int gm2_exchange_pack(const float* x, int64_t n, uint16_t* out, int64_t n_pad, void* stream) {
  return guarded([&] { launch_exchange_pack(x, n, (bf16_t*)out, n_pad, (hipStream_t)stream); });
}

int gm2_exchange_ranksum(const uint16_t* parts, int world, int64_t chunk, uint16_t* out, void* stream) {
  return guarded([&] { launch_exchange_ranksum((const bf16_t*)parts, world, chunk, (bf16_t*)out, (hipStream_t)stream); });
}

int gm2_exchange_unpack(const uint16_t* in, int64_t n, float* x, void* stream) {
  return guarded([&] { launch_exchange_unpack((const bf16_t*)in, n, x, (hipStream_t)stream); });
}

int gm2_grad_bucket_bounds(const gm2_dims* d, int64_t* lo_hi) {
  return guarded([&] { bucket_bounds(make_dims(d), lo_hi); });
}

int gm2_wait_grad_bucket(void* ws, int bucket, void* stream) {
  return with_ws(ws, [&](WsState& st) {
    if (bucket < 0 || bucket >= GM2_GRAD_BUCKETS) throw Gm2Error("bucket %d out of range", bucket);
    if (!st.recorded)
      throw Gm2Error("no gm2_train_fwd_bwd has recorded gradient buckets on this workspace (none has run, or "
                     "GM2_OPT_GRAD_BUCKETS is 0)");
    HIP_OK(hipStreamWaitEvent((hipStream_t)stream, st.bucket[st.bucket_ev[bucket]], 0));
  });
}

int gm2_set_option(int key, int value) {
  return guarded([&] { set_default_option(key, value); });
}

int gm2_get_option(int key, int* value) {
  return guarded([&] { *value = option_get(default_options(), key); });
}

int gm2_workspace_set_option(void* ws, int key, int value) {
  return guarded([&] { option_set(ws_state(ws).opt, key, value); });
}

int gm2_workspace_get_option(void* ws, int key, int* value) {
  return guarded([&] { *value = option_get(ws_state(ws).opt, key); });
}

int gm2_workspace_join(void* ws, void* stream) {
  return with_ws(ws, [&](WsState& st) { st.join((hipStream_t)stream); });
}

int gm2_workspace_set_collective(void* ws, gm2_allreduce_fn fn, void* user) {
  return guarded([&] {
    WsState& st = ws_state(ws);
    st.coll = fn;
    st.coll_user = user;
  });
}

int gm2_workspace_stat(void* ws, int key, int64_t* value) {
  return guarded([&] {
    if (!value) throw Gm2Error("null value");
    WsState& st = ws_state(ws);
    switch (key) {
      case GM2_STAT_SPLIT_DECODES:
      case GM2_STAT_EXACT_DECODES:
      case GM2_STAT_SPLIT_TILES:
      case GM2_STAT_EXACT_TILES:
      case GM2_STAT_BAND_ELEMENTS:
      case GM2_STAT_BAND_FLIPS:
      case GM2_STAT_BAND_OVERFLOW:
      case GM2_STAT_SINGLE_TILES:
      case GM2_STAT_OVERFLOW_TILES: {
        unsigned long long cum[8] = {}, ovf = 0;  // (the gated decodes' device counters: waits for the device)
        if (st.decode_cum) {
          HIP_OK(hipDeviceSynchronize());
          HIP_OK(hipMemcpy(cum, st.decode_cum, sizeof cum, hipMemcpyDeviceToHost));
          HIP_OK(hipMemcpy(&ovf, st.decode_ovf, sizeof ovf, hipMemcpyDeviceToHost));
        }
        switch (key) {
          case GM2_STAT_SPLIT_DECODES: *value = (int64_t)cum[5]; break;
          case GM2_STAT_EXACT_DECODES: *value = st.exact_decodes + (int64_t)cum[6]; break;
          case GM2_STAT_SPLIT_TILES: *value = (int64_t)cum[0]; break;
          case GM2_STAT_EXACT_TILES: *value = (int64_t)cum[1]; break;
          case GM2_STAT_BAND_ELEMENTS: *value = (int64_t)cum[2]; break;
          case GM2_STAT_BAND_FLIPS: *value = (int64_t)cum[3]; break;
          case GM2_STAT_SINGLE_TILES: *value = (int64_t)cum[7]; break;
          case GM2_STAT_OVERFLOW_TILES: *value = (int64_t)ovf; break;
          default: *value = (int64_t)cum[4]; break;
        }
        break;
      }
      default: throw Gm2Error("unknown statistic %d", key);
    }
  });
}

int gm2_workspace_release(void* ws) {
  bool dropped = false;
  const int rc = guarded([&] { dropped = ws_release(ws); });
  if (rc == 0 && dropped) {
    g_err = "gm2_workspace_release: a queued output-layer Adam update (GM2_OPT_DEFER_OUTPUT_ADAM) was discarded; "
            "call gm2_workspace_join before releasing to keep it";
    return 1;
  }
  return rc;
}

int gm2_timing_begin(int kernel_classes) {
  return guarded([&] { timing_begin(kernel_classes); });
}

int gm2_timing_end(double* total_ms, int64_t* launches) {
  return guarded([&] { timing_end(total_ms, launches); });
}

int gm2_timing_class(int kernel_class, double* total_ms, int64_t* launches) {
  return guarded([&] {
    if (!total_ms || !launches) throw Gm2Error("null output");
    timing_class(kernel_class, total_ms, launches);
  });
}

#ifdef GM2_DEBUG
// ---- debug build only (include/gm2_debug.h) ----
int gm2_debug_flags(unsigned* flags) {
  return guarded([&] {
    if (!flags) throw Gm2Error("null flags");
    *flags = dbg_take_kernels() | dbg_take_gemm() | dbg_take_masks();
  });
}

int gm2_debug_check_layout(const gm2_dims* d, int precision, int64_t* n_regions, int64_t* total) {
  return guarded([&] {
    const Layout o = make_layout(d, precision);
    auto r = t_regions;
    std::sort(r.begin(), r.end());
    int64_t end = 0;
    for (const auto& x : r) {
      if (x.first % 256) throw Gm2Error("region at %lld not 256-B aligned", (long long)x.first);
      if (x.first < end) throw Gm2Error("region at %lld overlaps the previous one (ends %lld)", (long long)x.first, (long long)end);
      end = x.first + x.second;
      if (end > o.total) throw Gm2Error("region at %lld (+%lld) past the total %lld", (long long)x.first, (long long)x.second, (long long)o.total);
    }
    // every named offset of the layout is one of the regions
    const int64_t named[] = {o.sE0, o.sE1, o.sE2, o.sHD, o.sD0, o.sD1, o.sD2, o.sD3, o.X, o.XB, o.HD, o.Z, o.dL,
                             o.slabs, o.side_slabs, o.DA, o.dH, o.AT5, o.dYT0, o.bnpart, o.colpart, o.losspart,
                             o.klpart, o.gradpart, o.colbwd, o.nahdr, o.nasq, o.clip, o.scal0, o.X1, o.XB1, o.syncb,
                             o.s3a, o.s3w, o.s3rn, o.s3cn, o.s3ctl, o.s3band, o.s3tlist, o.s3tcount, o.s3a1, o.s3w1,
                             o.s3ovf, o.s3bits, o.adamscal, o.ridx};
    auto known = [&](int64_t off) {
      for (const auto& x : r)
        if (x.first == off) return true;
      return false;
    };
    for (int64_t off : named)
      if (!known(off)) throw Gm2Error("named offset %lld is not a region start", (long long)off);
    for (int i = 0; i < 6; ++i)
      if (!known(o.Y[i]) || !known(o.A[i]) || !known(o.save[i]) || !known(o.dY[i]))
        throw Gm2Error("layer %d offsets are not region starts", i);
    if (n_regions) *n_regions = (int64_t)r.size();
    if (total) *total = o.total;
  });
}
#endif

}  // extern "C"
