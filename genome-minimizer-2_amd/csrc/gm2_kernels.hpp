// Internal kernel launchers of libgm2 (host side). Public C-ABI: include/gm2.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <stdexcept>
#include <string>

#include "gm2_common.hpp"

namespace gm2 {

struct Gm2Error : std::runtime_error {
  explicit Gm2Error(const std::string& s) : std::runtime_error(s) {}
  template <typename... A>
  Gm2Error(const char* fmt, A... a) : std::runtime_error(fmt_str(fmt, a...)) {}
  template <typename... A>
  static std::string fmt_str(const char* fmt, A... a) {
    char buf[512];
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wformat-security"
    snprintf(buf, sizeof buf, fmt, a...);
#pragma clang diagnostic pop
    return buf;
  }
};

#define GM2_CHECK_LAUNCH()                                                                     \
  do {                                                                                         \
    hipError_t e_ = hipGetLastError();                                                         \
    if (e_ != hipSuccess) throw ::gm2::Gm2Error("%s:%d launch: %s", __FILE__, __LINE__,       \
                                                hipGetErrorString(e_));                        \
  } while (0)

// indices into the per-step device scalar block (float[kNumScal]); written by the host
enum Scal {
  kScalBeta = 0,       // KL weight beta (loss_components.py:76-88)
  kScalWGamma = 1,     // weight * gamma of the gene-abundance term (0: component absent)
  kScalLambda = 2,     // lambda_l1 (0: component absent)
  kScalNegStep = 3,    // -lr / (1 - beta1^t)             (Adam step_size, negated)
  kScalBc2Sqrt = 4,    // sqrt(1 - beta2^t)
  kScalMaxNorm = 5,    // clip_grad_norm_ max_norm (<= 0: no clipping)
  kScalOneMinusB1 = 6, // 1 - beta1  (Adam: exp_avg.lerp_(grad, 1 - beta1))
  kScalBeta2 = 7,       // beta2       (exp_avg_sq.mul_(beta2).addcmul_(g, g, value=1 - beta2))
  kScalOneMinusB2 = 8,
  kScalAdamEps = 9,
  kScalNormAhead = 10,  // != 0: grads are as the last gm2_train_fwd_bwd wrote them (gm2.h GM2_S_NORM_AHEAD)
  kNumScal = 16
};

// C[M][N] = sum_k P(m, k) * Q(n, k). pk / qk: the operand is stored K-major ([rows][ld], K
// contiguous: P(m,k) = P[m*ld + k]) or MN-major ([K][ld]: P(m,k) = P[k*ld + m]). MN-major
// operands are read with ds_read_b64_tr_b16 (bf16) and need no transposed copy.
template <typename T>
struct GemmArgs {
  const T* P;
  int64_t ldp;
  const T* Q;
  int64_t ldq;
  int M, N, K;   // logical sizes (K already padded to 64, pads zero)
  int Mp, Np;    // padded M / N extents covered by the operand buffers (multiples of 128)
  int k_per_split;
  int pk = 1, qk = 1;
  // zero-copy batch rows (bf16 256x256 ping-pong plans only; GemmPlan must be tile 256): P's rows
  // (K-major P) or Q's k-rows (MN-major Q) are rows prow[m] / qrow[k] of the operand buffer instead
  // of m / k -- the input layer's GEMMs read the resident matrix's rows in place (gm2_batch.resident)
  const int32_t* prow = nullptr;
  const int32_t* qrow = nullptr;
  // rows of the buffer prow / qrow (and the loss epilogue's target rows) index: 0 = unknown (the
  // GM2_DEBUG build's bounds check then tests >= 0 only)
  int64_t idx_lim = 0;
};

// ---- tuning options (gm2.h GM2_OPT_*): results are bit-identical under every value ----
// Each workspace carries its own copy (gm2_workspace_set_option); gm2_set_option edits the process
// defaults that new workspaces and workspace-less calls (gm2_gemm) start from. The launchers read
// the options of the call in progress through opts(), which an OptionScope sets per C-ABI call.
struct Options {
  int gemm_pp = 1;       // GM2_OPT_GEMM_PP      ping-pong main loop of the 256x256 bf16 tiles
  int side_stream = 1;   // GM2_OPT_SIDE_STREAM  weight-gradient GEMMs on the workspace's side stream
  int recon_tile = 0;    // GM2_OPT_RECON_TILE   0 plan, 128 / 256 force
  int small_split = 1;   // GM2_OPT_SMALL_SPLIT  split-K of the chip-filling short-K 128-tile GEMMs
  int bn_epilogue = 1;   // GM2_OPT_BN_EPILOGUE  BatchNorm statistics in the GEMM store epilogue
  int small_waves = 8;   // GM2_OPT_SMALL_WAVES  waves of the 128x128 fp32-store tiles (4 or 8)
  int grid_cap = 3;      // GM2_OPT_GRID_CAP     capped grids: 1 dW9, 2 dWe0, 4 recon
  int input_chunks = 1;  // GM2_OPT_INPUT_CHUNKS launches of the input-layer weight gradient (1 or 4)
  int sync_bn = 0;       // GM2_OPT_SYNC_BN      train-mode BatchNorm over every rank's rows (collective)
  int defer_adam = 0;    // GM2_OPT_DEFER_OUTPUT_ADAM  output-layer Adam update beside the next step's hidden
                         //   layers on this many workgroups per CU (0 = not deferred)
  int grad_buckets = 1;  // GM2_OPT_GRAD_BUCKETS  record the gradient-bucket events (gm2_wait_grad_bucket)
  int sample_split = 1;  // GM2_OPT_SAMPLE_SPLIT  bf16x3 output layer of the sampling decode (bound permitting)
  int sample_single = 1; // GM2_OPT_SAMPLE_SINGLE the single-product bf16 tier of that gate (bound permitting)
  int band_cap = 65536;  // GM2_OPT_SAMPLE_BAND_CAP entries per band-list shard per decode (<= kBandShardCap;
                         //   smaller values exercise the overflow recompute)
  int single_bound_milli = 250;  // GM2_OPT_SAMPLE_SINGLE_BOUND the single tier's gate x 1000 (kSingleBound)
};
// validated edit of one option (throws on an unknown key or a bad value)
void option_set(Options& o, int key, int value);
int option_get(const Options& o, int key);
// process defaults: env GM2_GEMM_PP / GM2_SIDE_STREAM read once
Options default_options();
void set_default_option(int key, int value);
// the options of the C-ABI call in progress on this thread
const Options& opts();
struct OptionScope {
  explicit OptionScope(const Options& o);
  ~OptionScope();
  OptionScope(const OptionScope&) = delete;
  OptionScope& operator=(const OptionScope&) = delete;
  Options saved;
  int was;
};

// ---- live per-kernel timing (bench.py): hipEvent pairs around every launch of one class ----
enum KernelClass { kKcReconLoss = 1, kKcGemmStore = 2, kKcMask = 4, kKcAdam = 8 };
void timing_begin(int classes);
void timing_end(double* total_ms, int64_t* launches);
// the last timed region's total for one class (after timing_end)
void timing_class(int cls, double* total_ms, int64_t* launches);
struct TimedLaunch {  // records an event pair around a launch when its class is being timed
  TimedLaunch(int cls, hipStream_t s);
  ~TimedLaunch();
  int idx;
  hipStream_t s;
  int cls;
};

// ---- gemm.hip ----
// Options of the fp32 store epilogue (k_gemm_store): BatchNorm statistics of the stored tile, or
// a transposed store
struct StoreEpi {
  int mode = 0;             // 0 off; 1 forward (chunk mean, M2) of C; 2 backward (sum do, sum (y-mean) do)
  float2* part = nullptr;   // [row tile][ldp]
  int64_t ldp = 0;
  const float* Y = nullptr;  // mode 2: the layer's pre-BN output, row pitch ldy
  int64_t ldy = 0;
  const float* save = nullptr;  // mode 2: mean[H], invstd[H]
  const float* gamma = nullptr;
  const float* beta = nullptr;
  int H = 0;
  int trans = 0;  // store C^T: C0[n * ldc + m] (no bias, no statistics, one K pass)
  // one K pass only: sq[tile] = sum of the squares of the values the tile stored (fp64), tile =
  // (m0 / BM) * (Np / BN) + n0 / BN -- the clip-norm statistics of a weight gradient taken as it is
  // written (gm2_grad_norm with GM2_S_NORM_AHEAD)
  double* sq = nullptr;
  // > 0: the launch has fewer workgroups than tiles and each loops over tiles wg, wg + grid, ...
  // (grid = ceil(tiles / rounds) for the same number of rounds: the idle CUs of the last round
  // become free CUs for the other stream's work for the whole launch)
  int ntiles = 0;
};
// GEMM + BatchNorm statistics of its output in one launch when the plan allows (one K pass of
// 128-row tiles); returns false (nothing launched) otherwise
template <typename T>
bool launch_gemm_bn(const GemmArgs<T>& g, float* C, int64_t ldc, const float* bias, const StoreEpi& bn, hipStream_t s);
// C^T = (P . Q^T)^T into C [N][ldc] in one launch when the plan is one K pass; false otherwise
template <typename T>
bool launch_gemm_trans(const GemmArgs<T>& g, float* C, int64_t ldc, hipStream_t s, double* sq = nullptr);
// C = P . Q^T in one K pass with the per-tile sum of squares of C into sq (see StoreEpi::sq);
// false (nothing launched) when the plan splits K
template <typename T>
bool launch_gemm_sq(const GemmArgs<T>& g, float* C, int64_t ldc, double* sq, hipStream_t s, bool force_big = false);
// tiles of a one-pass launch of g (the sq entries it writes)
template <typename T>
int gemm_tiles(const GemmArgs<T>& g);

// splits < 0: use plan_gemm's split-K factor. Returns the number of slabs written.
template <typename T>
int launch_gemm_store(const GemmArgs<T>& g, int splits, float* C0, float* C1, int msplit, int64_t ldc,
                      int64_t slab, const float* bias, hipStream_t s);
template <typename T>
int gemm_recon_grid_blocks(const GemmArgs<T>& g);
template <typename T>
int gemm_recon_row_tiles(const GemmArgs<T>& g);

struct GemmPlan {
  int tile, splits;
};
template <typename T>
GemmPlan plan_gemm(const GemmArgs<T>& g);
// output layer GEMM computed transposed (P = W9 shadow [Gp][H], M = genes; Q = A5 [Bp][H], N =
// strains) + fused loss epilogue; xbits = row-major target bits [Bp][ldxb words]; dL [strain][ldd]
template <typename T>
void launch_gemm_recon_loss(const GemmArgs<T>& g, const float* bias, const uint32_t* xbits, int64_t ldxb, int with_grad,
                            const float* scal, T* dL, int64_t ldd, float* loss_part, float* colpart, int64_t ldcol,
                            hipStream_t s, const int32_t* xrows = nullptr);
// whether a GEMM with zero-copy rows (GemmArgs.prow / qrow) runs as planned: bf16, ping-pong main
// loop on, the 256x256 plan (and for qrow at most kMaxIdxRows k-rows per split)
constexpr int kMaxIdxRows = 8192;
template <typename T>
bool gemm_idx_ok(const GemmArgs<T>& g);
// The bf16x3 sampling decode's error bound (api.hip decode_split3): per logit at most
// kSplitUnit * ||a_r||_2 * ||w_g||_2 * 1.01 (Cauchy-Schwarz over the split's per-product error). The
// gate is per 256 x 256 tile: a tile runs split when kSplitUnit * max_r ||a_r|| * max_g ||w_g|| * 1.01
// over its 256 genome rows and 256 genes (the split kernels' block maxima) is <= kSplitBound, else
// the exact-fp32 kernel computes it.
// (kSplitBound sets what the split may cost, not what the masks are: every logit within the split's
// bound of the threshold is in the certified band and recomputed in fp64. Rounds 3-4 gated at
// 2.5e-4, from before the band recompute existed; a v1 checkpoint trained 10 epochs then ran no
// split tile at all (bench.py sample leg: 1.9 M genomes/s on the exact kernel). At 1e-3 the band
// stays small (tens of thousands of logits per 65,536-genome chunk on that checkpoint))
constexpr double kSplitBound = 1e-3;
constexpr double kSplitUnit = 4.62e-5;  // 3.02 x 2^-16, rounded up
constexpr int kSplitShards = 32;        // tile counters, sharded by blockIdx % kSplitShards
// The single-product tier (GM2_OPT_SAMPLE_SINGLE): one bf16 GEMM over the rounded operands (hi
// only, K = H) errs per logit by at most kSingleUnit * ||a_r|| ||w_g|| * 1.01 (each operand rounded
// to 8 significant bits: 2 x 2^-8 + 2^-16, rounded up). A tile takes it when kSingleUnit *
// max ||a_r|| * max ||w_g|| * 1.01 <= kSingleBound: its certified band is then ~170x the split's,
// i.e. more logits for the fp64 recompute, for a third of the split's MFMA work.
constexpr double kSingleBound = 0.25;
constexpr double kSingleUnit = 7.83e-3;
// Device-side choice of the output layer per 256 x 256 tile (every kernel launched over its full
// grid or a tile loop; a tile's workgroup runs only when the gate's verdict for its block is its
// `run`: 1 split, 2 exact, 3 single), counting the tiles it ran into tiles[blockIdx % 32]
struct MaskGate {
  const unsigned* ablk = nullptr;  // per 256-genome-row block: max ||a_r|| (fp32 bits)
  const unsigned* wblk = nullptr;  // per 256-gene block: max ||w_g|| (fp32 bits)
  int run = 0;
  unsigned* tiles = nullptr;
  int single = 0;                  // the single-product tier is on
  double single_bound = kSingleBound;
};
__device__ __forceinline__ int tile_level(const MaskGate& g, int m0, int n0) {
  const double a = (double)__uint_as_float(g.ablk[m0 >> 8]), w = (double)__uint_as_float(g.wblk[n0 >> 8]);
  if (g.single && kSingleUnit * a * w * 1.01 <= g.single_bound) return 3;
  return kSplitUnit * a * w * 1.01 <= kSplitBound ? 1 : 2;  // (NaN / inf: 2, the exact path)
}
// The certified band of the sampling decode (SURVEY.md 7 "Hard parts" (ii)): logits with
// |l - T| <= coef * ||a_r|| * ||w_g|| (T = the mask threshold) may sit on either side of T in the
// reference's own fp32 arithmetic; the mask epilogues append those (row, gene) pairs to a band list
// and k_band_fix recomputes each one's logit in fp64 from the same fp32 activations / weights and
// sets its mask bit from that.
//   coef (split tiles) = kSplitUnit * 1.01 + gamma_3H + gamma_H: the split's own error, its fp32
//     accumulation of 3H products and the reference's fp32 accumulation of H products
//   coef (exact tiles) = 2 gamma_H (gamma_n = n u / (1 - n u), u = 2^-24)
// The epilogues test |d| <= rmax * coef * ||w_g|| (1 + 2^-20) + 2^-21 (|b| + T), d = acc + b - T
// as they form it and rmax the largest of the four row norms a lane holds in one fragment: a
// superset of the band (the extra terms cover the rounding of d and of the product).
// Each flagged element goes to its tile's slots when the launch has them (tslots > 0: slot index
// from a counter in LDS, the tile's count stored once at the end of the tile; no global atomic on
// the common path), else (and for a tile's elements past its slots) to the list's kBandShards
// shards of `cap` entries (shard = blockIdx % kBandShards, each with its own counter: one atomic per
// wave per fragment position that holds band elements). An entry past a shard's capacity is not
// lost: its 256 x 256 block (genome rows r >> 8, genes g >> 8) is flagged once (oflag) and listed
// (olist), and k_band_tile_fix recomputes EVERY logit of each listed block in fp64 after the band
// fix, so a mask bit never stays as a bf16 tier decided it inside the band (round 6).
constexpr int kBandShards = 64;
constexpr unsigned kBandShardCap = 1u << 16;  // entries per shard per decode call (64 x 64 K x 8 B = 32 MB)
constexpr int kBandTileSlots = 256;           // per 256 x 256 tile (a trained model: ~2 per split, ~80 per single tile)
struct MaskBand {
  const float* rn = nullptr;  // ||a_r|| per genome row (nullptr: no band check)
  const float* cn = nullptr;  // ||w_g|| per gene
  float coef = 0.f;
  unsigned* counts = nullptr; // [kBandShards]
  uint2* list = nullptr;      // [kBandShards][cap] (row, gene)
  unsigned cap = 0;
  // overflow: per 256 x 256 block a flag word (zeroed by the caller), the flagged blocks' ids
  // (row block * obn + gene block; capacity = the block count, so it cannot overflow) and their count
  unsigned* oflag = nullptr;
  unsigned* olist = nullptr;
  unsigned* ocount = nullptr;
  int obn = 0;                // gene blocks per row block
  unsigned oblocks = 0;       // blocks in the grid (the flag / list capacity)
  uint2* tlist = nullptr;     // [tiles][tslots] (row, gene), tile = TileXY::t of the launch's grid
  unsigned* tcount = nullptr; // [tiles] the tile's band count, of which min(count, tslots) in its slots
                              // (zeroed by the caller; a tile's kernel writes its own)
  unsigned* tfound = nullptr; // [kBandShards] sum of the slot entries (statistics)
  int tslots = 0;
  // the single-product tier: a tile whose band exceeds its slots drops the rest (no shard entries)
  // and is re-run as bf16x3 in place (k_gemm_mask_tiered); its tile is then counted as split
  int drop_overflow = 0;
  unsigned* tiles_done = nullptr;  // [kSplitShards] tiles completed with drop_overflow (statistics)
};
inline double band_gamma(double n) { return n * 0x1p-24 / (1.0 - n * 0x1p-24); }
// the two bf16 tiers of the gated decode in one launch (gemm.hip k_gemm_mask_tiered): g1 / band1
// the single product (K = H), g3 / band3 the bf16x3 split (K' = 2H), gate3 the verdicts (run 1) and
// the split tiles' counter; gate1.tiles unused (band1.tiles_done counts the single tiles)
void launch_gemm_mask_tiered(const GemmArgs<bf16_t>& g1, const GemmArgs<bf16_t>& g3, const float* bias, uint8_t* mask,
                             int64_t ldm, uint8_t* bits, int64_t ldb, hipStream_t s, MaskGate gate1, MaskBand band1,
                             MaskGate gate3, MaskBand band3);
// k_band_fix over every shard's entries and every tile's slots: fp64 logit of (A[row], W[gene]) +
// bias, mask bit = (float)logit > T (the correctly rounded fp32 logit against the reference's
// threshold); packed bits (bits != nullptr) or u8 mask. flips: the bits it changed
void launch_band_fix(const MaskBand& band, int ntiles, const float* A, int64_t lda, const float* W, int64_t ldw,
                     const float* bias, int H, uint8_t* bits, int64_t ldb, uint8_t* mask, int64_t ldm, unsigned* flips,
                     hipStream_t s);
// k_band_tile_fix over the blocks band.olist lists (band.ocount of them, read on the device): every
// logit of rows [256 rb, min(256 rb + 256, n)) x genes [256 gb, min(.., G)) recomputed in fp64 as
// k_band_fix does, the block's mask bits rewritten (packed: whole 32-bit words; pad genes 0), flips
// counted. Launched after launch_band_fix on a fixed grid (nothing to do = one load per workgroup).
void launch_band_tile_fix(const MaskBand& band, const float* A, int64_t lda, const float* W, int64_t ldw,
                          const float* bias, int H, int n, int G, uint8_t* bits, int64_t ldb, uint8_t* mask,
                          int64_t ldm, unsigned* flips, hipStream_t s);
// one workgroup: the decode call's per-call counters -> the workspace's cumulative ones (DecodeCtl);
// ocount / ocum: the blocks k_band_tile_fix recomputed this call -> their cumulative count
// packed mask bits [n][ldb] (bit g % 8 of byte g / 8) -> u8 [n][ldm] (0 / 1), any row alignment
void launch_expand_bits(const uint8_t* bits, int64_t ldb, int n, int G, uint8_t* out, int64_t ldm, hipStream_t s);
void launch_decode_stats(const unsigned* tiles_split, const unsigned* tiles_exact, const unsigned* tiles_single,
                         const unsigned* counts, const unsigned* tfound, const unsigned* flips, unsigned cap,
                         unsigned long long* cum, const unsigned* ocount, unsigned long long* ocum, hipStream_t s);

// output layer + threshold (sampling / metrics): u8 mask, packed bits, probs, per-row (TP, FP, FN).
// big (bf16 only): the bf16x3 split decode -- 256x256 ping-pong tiles over operands in
// launch_split3's interleaved (hi | lo) layout, K = 2 x the hidden width, hi.hi + hi.lo + lo.hi
template <typename T>
void launch_gemm_mask(const GemmArgs<T>& g, const float* bias, uint8_t* mask, int64_t ldm, float* probs,
                      int64_t ldpr, hipStream_t s, uint8_t* bits = nullptr, int64_t ldb = 0, int* counts = nullptr,
                      const uint32_t* xbits = nullptr, int64_t ldxb = 0, float thr = 0.5f, bool big = false,
                      MaskGate gate = {}, MaskBand band = {});

// ---- kernels.hip ----
constexpr int kBnRowChunk = 128;  // rows per BatchNorm partial-statistics chunk
constexpr int kReparamRows = 16;  // batch rows per block of the reparameterisation kernels (their partials)

// gather strain rows of the resident u8 matrix into X [Bp][ldx] (T), plus the row-major bit-packed
// target [Bp][ldxb words] (bit g%32 of word g/32 of row b = X[b][g]) that the reconstruction-loss
// zero-copy rows: ridx[i] = rows[i] (or i when rows is null) for i < n, the resident matrix's zero
// row S for n <= i < nfill
void launch_resident_rows(const int32_t* rows, int n, int nfill, int64_t S, int32_t* ridx, hipStream_t s);
// epilogue reads; zero-fills columns >= G and rows >= B up to the padded extents
template <typename T>
void launch_gather_rows(const uint8_t* data, int64_t ld_data, const int32_t* rows, int B, int G, T* X, int64_t ldx,
                        int Gp, int Bp, uint32_t* xbits, int64_t ldxb, hipStream_t s);

// BN forward: y = sum of S slabs + bias -> Y; per-chunk (mean, M2) partials
void launch_bn_fwd_partial(const float* slabs, int S, int64_t slab, int64_t ld, const float* bias, int B, int H,
                           float* Y, float* part, hipStream_t s);
// BN backward: partials of sum(do), sum((y-mean)*do) with do = dA * [bn_out > 0]; optionally
// writes the summed split-K dA (dsum) so the apply pass reads one slab instead of S
void launch_bn_bwd_partial(const float* dslabs, int S, int64_t slab, const float* Y, int64_t ld, const float* save,
                           const float* gamma, const float* beta, int B, int H, float* part, float* dsum,
                           hipStream_t s);
// bf16x3 split of fp32 rows (the sampling decode's output layer): out [rows_pad][2K], each 64-column
// K-tile c = (hi | lo) of columns [32c, 32c + 32) (K % 32 == 0); rows >= rows zero; rn[r] = the row's
// 2-norm (rounded up; 0 for pad rows), blk[r / 256] = max of rn over each 256-row block (fp32 bits,
// atomic max: zero it first). rows_pad % 256 == 0.
void launch_split3(const float* X, int64_t ldx, int rows, int rows_pad, int K, bf16_t* out, int64_t ldo, float* rn,
                   unsigned* blk, hipStream_t s, bf16_t* out1 = nullptr);
// dst[c][r] = src[r][c] for an R x Cn block (multiples of 64)
template <typename T>
void launch_transpose(const T* src, int64_t lds_, int R, int Cn, T* dst, int64_t ldd, hipStream_t s);
// BatchNorm finalize (chunk merge per column) + elementwise apply in one launch per layer
// (sync != nullptr: SyncBN, the global batch's all-reduced sums from launch_bn_sync_pack)
template <typename T>
void launch_bn_fwd_apply(const float* Y, int64_t ld, const float* part, int B, int Bp, int H, int train,
                         const float* gamma, const float* beta, float* rmean, float* rvar, float* save, T* A,
                         hipStream_t s, const double* sync = nullptr);
template <typename T>
void launch_bn_bwd_apply(const float* da, const float* Y, int64_t ld, const float* part, int B, int Bp, int H,
                         int train, const float* save, const float* gamma, const float* beta, float* dgamma,
                         float* dbeta, T* dY, float* colpart, hipStream_t s, const double* sync = nullptr,
                         T* dYT = nullptr, int64_t ldt = 0);
// SyncBN: this rank's [sum | sum of squares (mode 0) or sum (y-mean)do (mode 1) | rows, 0] (2H + 2 doubles)
void launch_bn_sync_pack(const float* part, int B, int H, int mode, double* out, hipStream_t s);
// SyncBN, a rank with no rows: the running-statistics update from the all-reduced sums
void launch_bn_sync_running(const double* sync, int H, float* rmean, float* rvar, hipStream_t s);
// reparameterization + KL (model.py:100-104, loss_components.py:77)
template <typename T>
void launch_reparam(const float* slabs, int S, int64_t slab, int L, const float* bmu, const float* blv,
                    const float* eps, int B, int Bp, float* HD, T* Z, int64_t ldz, T* ZT, int64_t ldzt, int Lrows,
                    float* kl_part, hipStream_t s);
template <typename T>
void launch_reparam_bwd(const float* dzslabs, int S, int64_t slab, int64_t ldslab, const float* HD,
                        const float* eps, const float* scal, int B, int Bp, int L, T* dH, int64_t ldh,
                        const float* dmu_ext, const float* dlv_ext, float* colpart, hipStream_t s);
// z = mu + exp(lv/2)*eps over n elements (z != NULL), and/or its backward (dz != NULL -> dmu, dlv)
void launch_reparameterize(int64_t n, const float* mu, const float* lv, const float* eps, float* z, const float* dz,
                           float* dmu, float* dlv, hipStream_t s);
// dl = dp*(1-p)*p -> dL (T) [Bp][ldd] + per-64-row column partial sums [Bp/64][Gp]
template <typename T>
void launch_sigmoid_bwd(const float* p, const float* dp, int64_t ldp, int B, int Bp, int G, int Gp, T* dL, int64_t ldd,
                        float* colpart, hipStream_t s);
// out[n] = sum_r part[r*ld + n]  (deterministic order)
void launch_colsum(const float* part, int rows, int64_t ld, int64_t n, float* out0, float* out1, int64_t nsplit,
                   hipStream_t s);
// C0/C1 (row split at msplit) = sum of S split-K slabs [S][M][N] (slab stride `slab`)
void launch_slab_sum(const float* slabs, int S, int64_t slab, int M, int N, float* C0, float* C1, int msplit,
                     int64_t ldc, hipStream_t s);
// forward tail: loss[0..1] = sums of the output-layer tile partials (stride 2), loss[2] = sum of
// the KL partials; cout[c] (when non-null) = sum over `rows` of cpart[r][c]
// hdr (when non-null) <- {hv0, hv1}: the norm-ahead header of the training call (NormAhead)
void launch_fwd_tail(const float* lpart, int nl, const float* kpart, int nk, double* loss, const float* cpart, int rows,
                     int64_t ld, int64_t n, float* cout, int* hdr, int hv0, int hv1, hipStream_t s);

// bf16 gradient exchange (gm2.h gm2_exchange_*): fp32 -> bf16 (RNE, zero pad to n_pad); the rank-order
// fp32 sum of `world` bf16 chunks rounded to bf16 (chunk % 8 == 0); bf16 -> fp32
void launch_exchange_pack(const float* x, int64_t n, bf16_t* out, int64_t n_pad, hipStream_t s);
void launch_exchange_ranksum(const bf16_t* parts, int world, int64_t chunk, bf16_t* out, hipStream_t s);
void launch_exchange_unpack(const bf16_t* in, int64_t n, float* x, hipStream_t s);

// ---- masks.hip: consumers of the packed sampled masks ----
void launch_count_groups(const uint8_t* bits, int64_t n, int64_t ldb, const int32_t* goff, int64_t ngroups,
                         const int32_t* pos, int32_t* counts, hipStream_t s);
void launch_row_offsets(const uint8_t* bits, int64_t n, int64_t ldb, const uint8_t* keep, int64_t* offsets,
                        hipStream_t s);
void launch_compact(const uint8_t* bits, int64_t n, int64_t ldb, const uint8_t* keep, const int64_t* offsets,
                    int32_t* idx, hipStream_t s);

// parameter tensor table for the multi-tensor optimizer / shadow kernels
struct TensorDesc {
  int64_t off;        // offset in the flat fp32 param/grad/m/v buffers
  int64_t rows, cols;
  void* shadow;       // padded GEMM copy (T) [.. rows ..][sld] or nullptr
  int64_t sld;
  int64_t srow0;      // first shadow row of this tensor (mean/logvar share one shadow)
  void* shadowT;      // transposed padded copy [cols][tld] or nullptr
  int64_t tld;
  int64_t tile0;      // first 64x64 tile of this tensor in the shadow-sync grid
};
constexpr int kMaxTensors = 32;
struct TensorTable {
  int n;
  TensorDesc t[kMaxTensors];
};

template <typename T>
void launch_shadow_sync(const TensorTable& tt, const float* params, hipStream_t s);
// fused L1 + clip + Adam over the full 30-tensor table (tile0 = first 4096-element block of each
// tensor), writing natural-layout shadows of the tensors that have one; max_grid > 0 caps the
// workgroups (each then loops over blocks)
template <typename T>
void launch_adam_fused(const TensorTable& tt, const float* grads, float* params, float* m, float* v, const float* scal,
                       const float* clip, hipStream_t s, int max_grid = 0, float* scal_copy = nullptr);
// sum((g + lambda*sign(p))^2) and sum(|p|) over all params -> partials; then finalize
// Clip-norm statistics taken in the GEMM epilogues of the training call (StoreEpi::sq): hdr[0] = 1
// when both big weight gradients (input layer [lo0, hi0), output layer [lo9, hi9) of the flat
// buffer) were stored in one pass with their per-tile sums of squares in sq[0 .. hdr[1]). Used
// instead of re-reading those ranges when scal[kScalNormAhead] != 0 and there is no L1 term.
struct NormAhead {
  const int* hdr = nullptr;
  const double* sq = nullptr;
  int64_t lo0 = 0, hi0 = 0, lo9 = 0, hi9 = 0;
};
void launch_grad_stats(const float* params, const float* grads, int64_t n, const float* scal, double* part,
                       int nblocks, const NormAhead& na, hipStream_t s);
// clip coefficient / norm -> clip_out[0..1]; loss_slots (when non-null) [0] = sum |theta|, [1] = norm
void launch_grad_finalize(const double* part, int nblocks, const float* scal, float* clip_out,
                          double* loss_slots, const NormAhead& na, hipStream_t s);

int grad_stats_blocks(int64_t n);

#ifdef GM2_DEBUG
// read-and-clear the debug flag word of each translation unit (gm2_common.hpp DebugBit)
unsigned dbg_take_kernels();
unsigned dbg_take_gemm();
unsigned dbg_take_masks();
#endif

}  // namespace gm2
