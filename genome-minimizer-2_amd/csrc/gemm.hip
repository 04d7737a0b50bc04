// MFMA GEMM for the VAE hot path: C[M,N] = sum_k P[m,k] * Q[n,k]  ("NT": both operands
// K-contiguous, the layout the 16x16 MFMA fragments read with one ds_read_b128 per lane).
//
//  * T = bf16_t : v_mfma_f32_16x16x32_bf16 (training fast path, fp32 accumulate)
//  * T = float  : v_mfma_f32_16x16x4_f32   (exact-f32 path: sampling decode + parity training)
//
// Tile configurations (Cfg<BM, BN, WGM, WGN>): a block of WGM x WGN waves owns a BM x BN output
// tile, each wave a (BM/WGM) x (BN/WGN) sub-tile of 16x16 MFMA fragments.
//   Big   256x256, 8 waves (2x4, 128x64 per wave): the G x H GEMMs (half the L2->LDS bytes per
//         FLOP of a 128x128 tile, which at full MFMA rate would need ~36 TB/s of L2 bandwidth).
//   Small 128x128, 4 waves (2x2, 64x64 per wave): the H x H / latent GEMMs.
// One K-step = one 128-byte row chunk per operand row (64 bf16 / 32 f32). Operands are staged
// HBM->LDS with global_load_lds_dwordx4 (no VGPR round trip) into a 2-stage ring; the LDS image
// is XOR-swizzled (chunk ^= (row>>1)&7) through the per-lane SOURCE address, which makes the
// 16-lane ds_read_b128 groups conflict-free.
// Block -> tile: 1-D grid, bijective XCD remap (consecutive logical tiles share an XCD's L2),
// then split-K slice outermost and GROUP_M=8 grouped (m fastest) tile order.
//
// Contract (checked on the host): every operand buffer has >= roundup(M|N, tile) rows, K is a
// multiple of 64, pads are zero.
#include "gm2_common.hpp"
#include "gm2_kernels.hpp"

#include <atomic>
#include <cstdlib>
#include <map>
#include <mutex>
#include <set>
#include <type_traits>
#include <utility>
#include <vector>

namespace gm2 {

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// Diagnostic timestamps (s_memrealtime, 100 MHz) of the store kernel's phases per workgroup; only
// compiled into the standalone probe tools/stamp_gemm.hip, never into libgm2.
#ifdef GM2_STAMPS
__device__ unsigned long long g_stamp[16384][8];
#define GM2_STAMP(i) \
  if (threadIdx.x == 0) g_stamp[blockIdx.x][i] = __builtin_amdgcn_s_memrealtime()
#else
#define GM2_STAMP(i)
#endif

template <int BM_, int BN_, int WGM_, int WGN_, int NS_ = 2, int MINW_ = 1>
struct Cfg {
  static constexpr int MINW = MINW_;                 // min waves per SIMD (launch bounds: VGPR cap)
  static constexpr int BM = BM_, BN = BN_, WGM = WGM_, WGN = WGN_;
  static constexpr int NT = 64 * WGM * WGN;          // threads
  static constexpr int WTM = BM / WGM, WTN = BN / WGN;
  static constexpr int FM = WTM / 16, FN = WTN / 16;  // 16x16 fragments per wave
  static constexpr int STAGE = (BM + BN) * 128;      // bytes per pipeline stage
  static constexpr int NS = NS_;                     // pipeline stages in LDS
  static constexpr int LDS = NS * STAGE;
  static constexpr int LPS = (BM + BN) * 8 / NT;     // global_load_lds per thread per stage
};
using Big = Cfg<256, 256, 2, 4>;
using Small = Cfg<128, 128, 2, 2>;
// The fp32-output 128x128 tiles (hidden-layer GEMMs: one tile per CU, K = 1024 in 16 steps of
// ~0.2 us of MFMA each, against ~1 us from global_load_lds issue to landing): a 4-stage ring keeps
// three K-steps in flight instead of one.
using SmallDeep = Cfg<128, 128, 2, 2, 4>;
// The same tile with 8 waves (2x4, 64x32 each): two waves per SIMD, so one's LDS reads and waits
// hide behind the other's MFMAs (GM2_OPT_SMALL_WAVES = 8)
using SmallDeep8 = Cfg<128, 128, 2, 4, 4>;

struct TileXY {
  int m0, n0, split, t;
};

// XCD-aware, grouped tile order (see header)
__device__ __forceinline__ int xcd_wg(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}
__device__ __forceinline__ int xcd_wg() { return xcd_wg(blockIdx.x, gridDim.x); }

// logical tile t (GROUP_M = 8 supergroups, m fastest) -> tile origin
template <class C>
__device__ __forceinline__ TileXY tile_at(int t, int tm, int tn, int split) {
  constexpr int GROUP = 8;
  const int per_group = GROUP * tn;
  const int grp = t / per_group;
  const int first_m = grp * GROUP;
  const int gsize = min(tm - first_m, GROUP);
  const int in = t - grp * per_group;
  const int pm = first_m + in % gsize;
  const int pn = in / gsize;
  return {pm * C::BM, pn * C::BN, split, pm * tn + pn};
}

template <class C>
__device__ __forceinline__ TileXY tile_of(int tm, int tn) {
  const int wg = xcd_wg();
  const int ntile = tm * tn;
  const int split = wg / ntile;
  return tile_at<C>(wg - split * ntile, tm, tn, split);
}

// ---- operand staging (HBM -> LDS with global_load_lds_dwordx4; LDS destination lane-linear) ----
// K-major operand (stored [rows][ld], K contiguous): the tile is ROWS rows x 128 B (one K-step);
// 16-B chunk c of row r lives at chunk position c ^ ((r>>1)&7)  -> conflict-free ds_read_b128.
template <class C, typename T, int ROWS>
__device__ __forceinline__ void stage_kmajor(const T* __restrict__ P, int64_t ldp, int row0, int k0, char* lds,
                                             int wid, int lane) {
  constexpr int EPC = 16 / sizeof(T);
  constexpr int PER = ROWS * 8 / C::NT;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = j * C::NT + wid * 64 + lane;
    const int row = i >> 3;
    const int c = (i & 7) ^ ((row >> 1) & 7);
    const T* src = P + (int64_t)(row0 + row) * ldp + k0 + c * EPC;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds + (j * C::NT + wid * 64) * 16), 16, 0, 0);
  }
}

// MN-major operand (stored [K][ld], its M or N dimension contiguous): the tile is KT k-rows x
// R elements; 16-B chunk c of k-row k lives at chunk position c ^ swz(k). swz keeps chunk pairs
// together and spreads the 8 k-rows one 32-lane half of a ds_read_b64_tr_b16 touches over 8
// distinct 32-B bank groups (conflict-free transposed reads).
__device__ __forceinline__ int swz_mn(int k) { return 2 * ((k & 3) | ((k >> 1) & 4)); }

template <class C, typename T, int R>
__device__ __forceinline__ void stage_mnmajor(const T* __restrict__ P, int64_t ldp, int col0, int k0, char* lds,
                                              int wid, int lane) {
  constexpr int EPC = 16 / sizeof(T);
  constexpr int CPR = R / EPC;                // chunks per k-row
  constexpr int PER = E<T>::KT * CPR / C::NT;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = j * C::NT + wid * 64 + lane;
    const int k = i / CPR;
    const int c = (i % CPR) ^ swz_mn(k);
    const T* src = P + (int64_t)(k0 + k) * ldp + col0 + c * EPC;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds + (j * C::NT + wid * 64) * 16), 16, 0, 0);
  }
}

__device__ __forceinline__ int frag_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// bf16 fragment of operand rows [r0, r0+16) for k-substep s (32 k): lane l holds row r0 + (l&15),
// k = 32s + 8(l>>4) + j, j = 0..7 (the 16x16x32 MFMA A/B lane map).
template <bool KMAJ, int R>
__device__ __forceinline__ bf16x8 frag_bf16(const char* tile, int r0, int s, int lane) {
  if constexpr (KMAJ) {
    return *(const bf16x8*)(tile + frag_off(r0 + (lane & 15), s * 4 + (lane >> 4)));
  } else {
    constexpr int RB = R * 2;  // bytes per k-row
    const int i = lane & 15, q = i >> 2, p = i & 3;
    const int k = s * 32 + 8 * (lane >> 4) + q;
    const int c = (r0 >> 3) + (p >> 1);
    const char* a1 = tile + k * RB + ((c ^ swz_mn(k)) << 4) + (p & 1) * 8;
    const char* a2 = tile + (k + 4) * RB + ((c ^ swz_mn(k + 4)) << 4) + (p & 1) * 8;
    const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a1);
    const bf16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a2);
    return bf16x8{v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
  }
}

// f32 fragment for k-substep s (16 k): lane l holds row r0 + (l&15), k = 16s + 4(l>>4) + j, j = 0..3
template <bool KMAJ, int R>
__device__ __forceinline__ f32x4 frag_f32(const char* tile, int r0, int s, int lane) {
  if constexpr (KMAJ) {
    return *(const f32x4*)(tile + frag_off(r0 + (lane & 15), s * 4 + (lane >> 4)));
  } else {
    constexpr int RB = R * 4;
    const int r = r0 + (lane & 15);
    f32x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = s * 16 + 4 * (lane >> 4) + j;
      v[j] = *(const float*)(tile + k * RB + (((r >> 2) ^ swz_mn(k)) << 4) + (r & 3) * 4);
    }
    return v;
  }
}

// Wait until at most `r` (0 <= r <= NS - 2; negative = 0) later stages' loads are in flight.
template <class C>
__device__ __forceinline__ void wait_stages(int r) {
  static_assert(C::NS <= 5 && 3 * C::LPS <= 63, "vmcnt range");
  if (C::NS >= 5 && r >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * C::LPS) : "memory");
  else if (C::NS >= 4 && r >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * C::LPS) : "memory");
  else if (C::NS >= 3 && r >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::LPS) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Main loop. acc[mi][ni][j] = C[m0 + wm*WTM + mi*16 + 4*(lane>>4) + j][n0 + wn*WTN + ni*16 + (lane&15)]
// AK / BK: P / Q stored K-major (true) or MN-major (false).
template <class C, typename T, bool AK, bool BK>
__device__ __forceinline__ void mainloop(const T* __restrict__ P, int64_t ldp, const T* __restrict__ Q, int64_t ldq,
                                         int m0, int n0, int kbeg, int nk, char* smem,
                                         f32x4 (&acc)[C::FM][C::FN]) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / C::WGN, wn = wid % C::WGN;
  constexpr int KT = E<T>::KT;
#pragma unroll
  for (int a = 0; a < C::FM; ++a)
#pragma unroll
    for (int b = 0; b < C::FN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nk <= 0) return;

  auto stage = [&](char* buf, int k0) {
    if constexpr (AK) stage_kmajor<C, T, C::BM>(P, ldp, m0, k0, buf, wid, lane);
    else stage_mnmajor<C, T, C::BM>(P, ldp, m0, k0, buf, wid, lane);
    if constexpr (BK) stage_kmajor<C, T, C::BN>(Q, ldq, n0, k0, buf + C::BM * 128, wid, lane);
    else stage_mnmajor<C, T, C::BN>(Q, ldq, n0, k0, buf + C::BM * 128, wid, lane);
  };
  // NS-stage ring: K-step kt lives in buffer kt % NS; step kt + NS - 1 is issued at the top of
  // step kt into the buffer step kt - 1 used (every wave passed the barrier after reading it).
  // The wait at the end of step kt lets the stages after kt + 1 stay in flight (counted vmcnt).
  constexpr int NS = C::NS;
#pragma unroll
  for (int st = 0; st < NS - 1; ++st)
    if (st < nk) stage(smem + st * C::STAGE, kbeg + st * KT);
  wait_stages<C>(min(NS - 2, nk - 1));
  __syncthreads();
  GM2_STAMP(1);

  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt % NS) * C::STAGE;
    if (kt + NS - 1 < nk) stage(smem + ((kt + NS - 1) % NS) * C::STAGE, kbeg + (kt + NS - 1) * KT);
    const char* sA = cur;
    const char* sB = cur + C::BM * 128;
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 b[C::FN];
#pragma unroll
        for (int ni = 0; ni < C::FN; ++ni) b[ni] = frag_bf16<BK, C::BN>(sB, wn * C::WTN + ni * 16, s, lane);
#pragma unroll
        for (int mi = 0; mi < C::FM; ++mi) {
          const bf16x8 a = frag_bf16<AK, C::BM>(sA, wm * C::WTM + mi * 16, s, lane);
#pragma unroll
          for (int ni = 0; ni < C::FN; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[ni], acc[mi][ni], 0, 0, 0);
        }
      }
    } else {
      // exact-fp32 path: each K-step's 32 products go into a fresh partial sum that is then added
      // to the accumulator, so a K-long dot product is a chain of K/32 additions of 32-term blocks
      // instead of one K-long fma chain. On the long-K GEMMs of the step (K = G = 55,040, the input
      // layer and the output layer's input gradient) this keeps the rounding error of the train-mode
      // BatchNorm backward's near-cancelling column sums at the level of the reference's own MKL
      // arithmetic (tools/diag/c3_chain.py: the single chain was 2.5-6x worse on the hidden layers)
      f32x4 part[C::FM][C::FN];
#pragma unroll
      for (int a = 0; a < C::FM; ++a)
#pragma unroll
        for (int b = 0; b < C::FN; ++b) part[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        f32x4 b[C::FN];
#pragma unroll
        for (int ni = 0; ni < C::FN; ++ni) b[ni] = frag_f32<BK, C::BN>(sB, wn * C::WTN + ni * 16, s, lane);
#pragma unroll
        for (int mi = 0; mi < C::FM; ++mi) {
          const f32x4 a = frag_f32<AK, C::BM>(sA, wm * C::WTM + mi * 16, s, lane);
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int ni = 0; ni < C::FN; ++ni)
              part[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[ni][j], part[mi][ni], 0, 0, 0);
        }
      }
#pragma unroll
      for (int mi = 0; mi < C::FM; ++mi)
#pragma unroll
        for (int ni = 0; ni < C::FN; ++ni) acc[mi][ni] += part[mi][ni];
    }
    wait_stages<C>(min(NS - 2, nk - 2 - kt));
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// Ping-pong main loop for the 256x256 bf16 tile (8 waves = two groups of four, one wave of each
// group per SIMD). Each K-tile (64 k) is consumed in 4 phases, one 64x32 quadrant of each wave's
// 128x64 sub-tile per phase (16 MFMAs): (a0,b0) (a0,b1) (a1,b0) (a1,b1), where a = which 64 of
// the wave's 128 rows and b = which 32 of its 64 columns. The stage of a K-tile is split into the
// four matching half-tiles, each its own 16 KB LDS region of the tile's buffer:
//   A_a : the rows {g*128 + a*64 + 0..63 : g = 0,1}   (both groups' a-halves)
//   B_b : the cols {w*64 + b*32 + 0..31 : w = 0..3}
// Phase p of tile t: [L] ds_read this quadrant's new fragments from buffer t&1, [G] issue one
// half-tile into buffer (t+1)&1 (A0, B0, B1, A1 of tile t+1 at p = 0..3; with kPPDeep, the
// default, B1(t+1), A1(t+1), A0(t+2), B0(t+2): each half-tile as early as the WAR rule allows),
// [W] counted vmcnt, barrier, MFMAs, barrier. Group 1 runs one barrier behind group 0, so on every SIMD one wave
// computes while the other reads LDS and issues loads (MI355X_MICROARCH.md "Two waves per SIMD").
// Ordering (barrier instances counted globally, phase n = 4t+p):
//  * RAW: a half-tile issued at phase n_i is covered by every wave's vmcnt at phase n_w and read
//    at phase >= n_w + 1: A0(t+1), B0(t+1) retired at 4t+3, read at 4(t+1); B1 issued 4t+2,
//    retired 4t+4, read 4t+5; A1 issued 4t+3, retired 4t+5, read 4t+6. Steady-state wait
//    vmcnt(4) = two later half-tiles x 2 loads per thread; none at p = 2.
//  * WAR: a region of buffer (t+1)&1 is restaged >= 4 phases after its last read in tile t-1
//    (the rule needs >= 2).
// ---------------------------------------------------------------------------------------------
// mainloop_pp issues each half-tile two phases earlier (DEEP below): 4-5 phases between issue and
// retire instead of 2-3, 8 loads in flight -- the 256-tile kernels are bound by that latency, not
// by their barriers or L2 -> LDS bytes (profiles/r04_pp_deep_prefetch_ab.txt: -50 us/step)
constexpr bool kPPDeep = true;
namespace pp {
constexpr int REGION = 128 * 128;  // bytes of one half-tile region (128 rows x 128 B, or 64 k x 256 B)
constexpr int BUF = 4 * REGION;    // one K-tile: A0, A1, B0, B1
__device__ __forceinline__ int a_row(int r, int a) { return (r >> 6) * 128 + a * 64 + (r & 63); }
__device__ __forceinline__ int b_row(int r, int b) { return (r >> 5) * 64 + b * 32 + (r & 31); }

// one half-tile: 1024 16-B chunks, 2 per thread (lane-linear LDS destination, swizzled source).
// IDX (zero-copy rows): the thread's two rows (K-major) / k-rows (MN-major), j = 0, 1, are rr[j],
// read from the tile's LDS index table ahead of the issuing phase (idx_rows below)
template <bool KMAJ, bool ISA, bool IDX = false>
__device__ __forceinline__ void stage_half(const bf16_t* __restrict__ P, int64_t ld, int base, int half, int k0,
                                           char* region, int tid, const int* rr = nullptr) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int i = j * 512 + tid;
    const bf16_t* src;
    if constexpr (KMAJ) {
      const int row = i >> 3;
      const int c = (i & 7) ^ ((row >> 1) & 7);
      const int g = ISA ? a_row(row, half) : b_row(row, half);
      const int64_t r = IDX ? (int64_t)rr[j] : (int64_t)(base + g);
      src = P + r * ld + k0 + c * 8;
    } else {
      const int k = i >> 4;
      const int e = ((i & 15) ^ swz_mn(k)) * 8;
      const int g = ISA ? a_row(e, half) : b_row(e, half);
      const int64_t r = IDX ? (int64_t)rr[j] : (int64_t)(k0 + k);
      src = P + r * ld + base + g;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(region + (j * 512 + (tid & ~63)) * 16), 16, 0, 0);
  }
}

// the table entries of the thread's two rows of a K-major half-tile (tile-local rows a_row(.)) or
// of its two k-rows of an MN-major half-tile of K-tile t (table = the split's k-rows)
template <bool KMAJ>
__device__ __forceinline__ void idx_rows(const int* sidx, int half, int t, int tid, int (&rr)[2]) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int i = j * 512 + tid;
    if constexpr (KMAJ) rr[j] = sidx[a_row(i >> 3, half)];
    else rr[j] = sidx[t * 64 + (i >> 4)];
  }
}

__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}
}  // namespace pp

// S3 (the bf16x3 split decode): both operands in launch_split3's layout -- K-substep s = 0 of each
// K-tile is the hi part, s = 1 the lo part of the same 32 k -- and each fragment pair contributes
// hi.hi + hi.lo + lo.hi (three MFMAs instead of the two of a plain K-tile; lo.lo is dropped)
template <bool AK, bool BK, int IDX = 0, bool S3 = false>
__device__ __forceinline__ void mainloop_pp(const bf16_t* __restrict__ P, int64_t ldp, const bf16_t* __restrict__ Q,
                                            int64_t ldq, int m0, int n0, int kbeg, int nk, char* smem,
                                            f32x4 (&acc)[8][4], const int* sidx = nullptr) {
  // DEEP: the longer-prefetch issue order
  constexpr bool DEEP = kPPDeep;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // wave-uniform in an SGPR: the stagger barriers below must be branched around, not exec-masked
  const int wm = __builtin_amdgcn_readfirstlane(wid >> 2), wn = wid & 3;
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nk <= 0) return;
  // half-tile h (0 = A0, 1 = B0, 2 = B1, 3 = A1) of K-tile t -> its region
  auto region = [&](int t, int h) -> char* {
    const int off = h == 0 ? 0 : h == 3 ? 1 : h + 1;  // A0 0, A1 1, B0 2, B1 3
    return smem + (t & 1) * pp::BUF + off * pp::REGION;
  };
  // zero-copy rows: IDX 1 = P's rows (the tile's A rows: fixed, held for the tile), IDX 2 = Q's
  // k-rows (read one phase ahead of the two B-half issues of each K-tile, so the table read never
  // waits behind the phase's fragment reads)
  int ra0[2] = {0, 0}, ra1[2] = {0, 0}, rq[2] = {0, 0};
  if constexpr (IDX == 1) {
    pp::idx_rows<true>(sidx, 0, 0, tid, ra0);
    pp::idx_rows<true>(sidx, 1, 0, tid, ra1);
  }
  auto issue = [&](int t, int h) {
    const int k0 = kbeg + t * 64;
    char* r = region(t, h);
    if (h == 0 || h == 3) pp::stage_half<AK, true, IDX == 1>(P, ldp, m0, h == 0 ? 0 : 1, k0, r, tid, h == 0 ? ra0 : ra1);
    else pp::stage_half<BK, false, IDX == 2>(Q, ldq, n0, h == 1 ? 0 : 1, k0, r, tid, rq);
  };
  bf16x8 fa[4][2], fb0[2][2], fb1[2][2];
  auto read_a = [&](int t, int a) {
    const char* r = region(t, a == 0 ? 0 : 3);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int s = 0; s < 2; ++s) fa[mi][s] = frag_bf16<AK, 128>(r, wm * 64 + mi * 16, s, lane);
  };
  auto read_b = [&](int t, int b, bf16x8 (&fb)[2][2]) {
    const char* r = region(t, b == 0 ? 1 : 2);
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int s = 0; s < 2; ++s) fb[ni][s] = frag_bf16<BK, 128>(r, wn * 32 + ni * 16, s, lane);
  };
  auto mma = [&](int a, int b, const bf16x8 (&fb)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        f32x4& c = acc[a * 4 + mi][b * 2 + ni];
        if constexpr (S3) {
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mi][0], fb[ni][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mi][0], fb[ni][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mi][1], fb[ni][0], c, 0, 0, 0);
        } else {
#pragma unroll
          for (int s = 0; s < 2; ++s) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mi][s], fb[ni][s], c, 0, 0, 0);
        }
      }
    __builtin_amdgcn_s_setprio(0);
  };
  // prologue: all four half-tiles of tile 0; A0, B0 retired before the first reads
  if constexpr (IDX == 2) pp::idx_rows<false>(sidx, 0, 0, tid, rq);
  if constexpr (DEEP) {  // tile 0, then A0 and B0 of tile 1 (issued at phases 2 and 3 of tile -1)
#pragma unroll
    for (int h = 0; h < 4; ++h) issue(0, h);
    if (nk > 1) {
      issue(1, 0);
      if constexpr (IDX == 2) pp::idx_rows<false>(sidx, 0, 1, tid, rq);
      issue(1, 1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // A0(0), B0(0)
    } else {
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
  } else {
#pragma unroll
    for (int h = 0; h < 4; ++h) issue(0, h);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  }
  pp::barrier();
  GM2_STAMP(1);
  if (wm == 1) pp::barrier();  // stagger: group 1 one barrier behind
  if constexpr (DEEP) {
    // Issue order two phases earlier than below (each half-tile as soon as the WAR rule allows):
    // tile t issues B1(t+1) at phase 0, A1(t+1) at 1, A0(t+2) at 2, B0(t+2) at 3, so every half-tile
    // has four to five phases between its issue and its retire (two to three below). Retire points
    // are unchanged: B1(t) at phase 0, A1(t) at 1, A0 / B0 (t+1) at 3; 8 loads stay in flight.
    int rq2[2] = {0, 0};  // IDX 2: the k-rows of B0(t+2), read at phase 1
    for (int t = 0; t < nk; ++t) {
      const bool m1 = t + 1 < nk, m2 = t + 2 < nk;
      if constexpr (IDX == 2) {
        if (m1) pp::idx_rows<false>(sidx, 0, t + 1, tid, rq);  // B1(t+1)
      }
      // phase 0: (a0, b0)
      read_a(t, 0);
      read_b(t, 0, fb0);
      if (m1) {
        issue(t + 1, 2);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // retires B1(t)
      } else {
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      }
      pp::barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mma(0, 0, fb0);
      pp::barrier();
      // phase 1: (a0, b1)
      read_b(t, 1, fb1);
      if constexpr (IDX == 2) {
        if (m2) pp::idx_rows<false>(sidx, 0, t + 2, tid, rq2);
      }
      if (m1) {
        issue(t + 1, 3);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // retires A1(t)
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      pp::barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mma(0, 1, fb1);
      pp::barrier();
      // phase 2: (a1, b0)
      read_a(t, 1);
      if (m2) issue(t + 2, 0);
      pp::barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mma(1, 0, fb0);
      pp::barrier();
      // phase 3: (a1, b1)
      if (m2) {
        if constexpr (IDX == 2) {
          rq[0] = rq2[0];
          rq[1] = rq2[1];
        }
        issue(t + 2, 1);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // retires A0(t+1), B0(t+1)
      } else if (m1) {
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      }
      pp::barrier();
      __builtin_amdgcn_sched_barrier(0);
      mma(1, 1, fb1);
      pp::barrier();
    }
  } else {
    for (int t = 0; t < nk; ++t) {
      const bool more = t + 1 < nk;
      if constexpr (IDX == 2) {
        if (more) pp::idx_rows<false>(sidx, 0, t + 1, tid, rq);
      }
      // phase 0: (a0, b0)
      read_a(t, 0);
      read_b(t, 0, fb0);
      if (more) {
        issue(t + 1, 0);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // retires B1(t)
      } else {
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      }
      pp::barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mma(0, 0, fb0);
      pp::barrier();
      // phase 1: (a0, b1)
      read_b(t, 1, fb1);
      if (more) {
        issue(t + 1, 1);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // retires A1(t)
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      pp::barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mma(0, 1, fb1);
      pp::barrier();
      // phase 2: (a1, b0)
      read_a(t, 1);
      if (more) issue(t + 1, 2);
      pp::barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mma(1, 0, fb0);
      pp::barrier();
      // phase 3: (a1, b1)
      if (more) {
        issue(t + 1, 3);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // retires A0(t+1), B0(t+1)
      }
      pp::barrier();
      __builtin_amdgcn_sched_barrier(0);
      mma(1, 1, fb1);
      pp::barrier();
    }
  }
  if (wm == 0) pp::barrier();  // re-align the groups
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// ---------------------------------------------------------------------------------------------
// Epilogue 1: fp32 store. Rows m < msplit go to C0, rows >= msplit to C1 (row m - msplit); the
// split-K slice z writes slab z (C0 + z*slab). Optional per-column bias.
// ---------------------------------------------------------------------------------------------
//
// Optional BatchNorm statistics of the stored tile (bn.mode != 0; 128-row tiles, one K pass, no
// row split -- the host checks): per (128-row chunk = row tile, column) partials in the format of
// k_bn_fwd_partial / k_bn_bwd_partial, so the separate statistics pass over Y / dA disappears.
//   mode 1 (forward): v = acc + bias -> (chunk mean, M2), from sums of v - shift in fp32 with the
//           shift = the tile's first row (stable: the shift is a sample of the column).
//   mode 2 (backward): acc = dA; do = dA * [y*alpha + beta' > 0] with y read from bn.Y ->
//           (sum do, sum (y - mean) do).
// The store loop visits 4 fixed columns per thread, so the sums stay in registers and the threads
// of a column are combined through LDS once at the end.
__device__ __forceinline__ double sq4(float a, float b, float c, float d) {
  return ((double)a * a + (double)b * b) + ((double)c * c + (double)d * d);
}

template <class C, typename T, bool AK, bool BK, bool PP, int IDX, int EPI>
__device__ __forceinline__ void store_tile(const TileXY tl, const GemmArgs<T>& g, float* __restrict__ C0,
                                           float* __restrict__ C1, int msplit, int64_t ldc, int64_t slab,
                                           const float* __restrict__ bias, const StoreEpi& bn, char* smem);

// IDX (zero-copy rows, PP only): 1 = P's rows through g.prow, 2 = Q's k-rows through g.qrow; the
// tile's slice of the index array sits in an LDS table after the staging ring
// EPI (the epilogue, fixed at compile time for the 256x256 kernels so each instantiation carries only
// its own store code: with the general one every 256x256 kernel spilled 12-21 VGPRs, with these
// none): 0 = general (bias, BatchNorm statistics, row split, unaligned rows, transposed store),
// 1 = plain fp32 store (split-K slabs or one pass, rows aligned or not, optional per-tile sums of
// squares), 2 = the transposed store straight from the accumulators (+ sums of squares), 3 = the
// transposed store through the LDS image (+ sums of squares)
template <class C, typename T, bool AK, bool BK, bool PP, int IDX = 0, int EPI = 0>
__global__ __launch_bounds__(C::NT, C::MINW) void k_gemm_store(GemmArgs<T> g, float* __restrict__ C0, float* __restrict__ C1,
                                                    int msplit, int64_t ldc, int64_t slab,
                                                    const float* __restrict__ bias, StoreEpi bn) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  GM2_STAMP(0);
  const int tm = g.Mp / C::BM, tn = g.Np / C::BN;
  if (bn.ntiles == 0) {  // one tile per workgroup
    store_tile<C, T, AK, BK, PP, IDX, EPI>(tile_of<C>(tm, tn), g, C0, C1, msplit, ldc, slab, bias, bn, smem);
    return;
  }
  // capped grid (one K pass): workgroup wg takes logical tiles wg, wg + grid, ... (every wave of
  // the block runs the same trip count; the LDS is reused after a barrier)
  const int ntile = tm * tn;
  for (int t = xcd_wg(); t < bn.ntiles; t += gridDim.x) {
    __syncthreads();
    store_tile<C, T, AK, BK, PP, IDX, EPI>(tile_at<C>(t % ntile, tm, tn, t / ntile), g, C0, C1, msplit, ldc, slab, bias,
                                      bn, smem);
  }
}

template <class C, typename T, bool AK, bool BK, bool PP, int IDX, int EPI>
__device__ __forceinline__ void store_tile(const TileXY tl, const GemmArgs<T>& g, float* __restrict__ C0,
                                           float* __restrict__ C1, int msplit, int64_t ldc, int64_t slab,
                                           const float* __restrict__ bias_in, const StoreEpi& bn, char* smem) {
  // (the specialised epilogues: their options fixed, so the general code below folds away)
  const float* __restrict__ bias = EPI == 0 ? bias_in : nullptr;
  const int bmode = EPI == 0 ? bn.mode : 0;
  const int btrans = EPI == 0 ? bn.trans : EPI >= 2;
  const int kbeg = tl.split * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  const int nk = (kend - kbeg) / E<T>::KT;
  GM2_DBG(tl.m0 + C::BM <= g.Mp && tl.n0 + C::BN <= g.Np && kbeg >= 0 && kend <= g.K, kDbgTile);
  f32x4 acc[C::FM][C::FN];
  if constexpr (PP) {
    int* sidx = (int*)(smem + C::LDS);
    if constexpr (IDX == 1) {
      for (int i = threadIdx.x; i < C::BM; i += C::NT) {
        sidx[i] = g.prow[tl.m0 + i];
        GM2_DBG(sidx[i] >= 0 && (g.idx_lim == 0 || sidx[i] < g.idx_lim), kDbgGemmIdx);
      }
      __syncthreads();
    } else if constexpr (IDX == 2) {
      for (int i = threadIdx.x; i < kend - kbeg; i += C::NT) {
        sidx[i] = g.qrow[kbeg + i];
        GM2_DBG(sidx[i] >= 0 && (g.idx_lim == 0 || sidx[i] < g.idx_lim), kDbgGemmIdx);
      }
      __syncthreads();
    }
    mainloop_pp<AK, BK, IDX>(g.P, g.ldp, g.Q, g.ldq, tl.m0, tl.n0, kbeg, nk, smem, acc, sidx);
  } else {
    static_assert(IDX == 0, "zero-copy rows: ping-pong main loop only");
    mainloop<C, T, AK, BK>(g.P, g.ldp, g.Q, g.ldq, tl.m0, tl.n0, kbeg, nk, smem, acc);
  }
  GM2_STAMP(2);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wm = wid / C::WGN, wn = wid % C::WGN;
  float* Cz = C0 + (int64_t)tl.split * slab;
  // Stage one 64-row band of the tile at a time through the (now free) staging LDS (row pitch
  // BN + 4 floats: the accumulator writes of lanes 16 apart land 16 banks apart), then store whole
  // rows with 16-byte stores (4 columns per thread; scalar where C's rows are not 16-B aligned or
  // at the N edge).
  // Transposed store (btrans): 16 lanes write 4 consecutive m each of one column n (256
  // contiguous bytes of C^T's row n), reading the image down a column (odd pitch: conflict-free).
  float* img = (float*)smem;
  const int pitch = btrans ? C::BN + 1 : C::BN + 4;
  constexpr int BR = 64, NBANDS = C::BM / BR, BPW = C::WTM / BR;  // bands, bands per wave row
  static_assert(BR * (C::BN + 4) * 4 <= C::LDS, "epilogue band must fit the staging LDS");
  constexpr int TPR = C::BN / 4, RPI = C::NT / TPR;  // threads per row, rows per pass
  static_assert(C::NT % TPR == 0 && BR % RPI == 0 && 2 * C::NT * 16 <= C::LDS, "epilogue shape");
  const int cq = (threadIdx.x % TPR) * 4, rq = threadIdx.x / TPR;
  const int n = tl.n0 + cq;
  const bool vec = ((ldc | slab) & 3) == 0 && ((((uintptr_t)C0) | ((uintptr_t)C1)) & 15) == 0;
  // Rows that are not 16-B aligned (ldc % 4 != 0, e.g. the [H][G] input-layer gradient at odd G):
  // row m's elements go into the image shifted by e_m = (address of (m, n0) in floats) % 4, so
  // every image chunk of 4 is one aligned 16-B global chunk; only the two end chunks of a row are
  // partial. e_m depends on the row only through m % 4 (j of the accumulator layout).
  const bool shiftvec = !vec && slab == 0 && !bias && bmode == 0 && !btrans && msplit >= g.M &&
                        (((uintptr_t)C0) & 3) == 0;
  const int e_base = (int)(((uintptr_t)(C0 + (int64_t)tl.m0 * ldc + tl.n0) >> 2) & 3), l3 = (int)(ldc & 3);
  float bb[4], sa[4], sb[4], sh[4], bmean[4], balpha[4], bbeta[4];
  double sqa = 0.0;  // sum of squares of the stored values (bn.sq), fp64 like the re-reading pass
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    bb[u] = (bias && n + u < g.N) ? bias[n + u] : 0.f;
    sa[u] = sb[u] = sh[u] = bmean[u] = balpha[u] = bbeta[u] = 0.f;
    if (bmode == 2 && n + u < g.N) {
      bmean[u] = bn.save[n + u];
      balpha[u] = bn.save[bn.H + n + u] * bn.gamma[n + u];
      bbeta[u] = fmaf(-bmean[u], balpha[u], bn.beta[n + u]);
    }
  }
  // Transposed store straight from the accumulators (bn.trans_direct): lane l of fragment (mi, ni)
  // holds rows m .. m + 3 (j) of column n, i.e. 16 contiguous bytes of C^T's row n -- one 16-B store
  // per fragment, no LDS image and no barriers (each instruction writes 16 rows x 64 B; the L2 merges
  // the two halves of each 128-B line, written by consecutive fragments)
  const bool direct = EPI == 2;
  if (direct) {
#pragma unroll
    for (int mi = 0; mi < C::FM; ++mi)
#pragma unroll
      for (int ni = 0; ni < C::FN; ++ni) {
        const int nn = tl.n0 + wn * C::WTN + ni * 16 + (lane & 15);
        const int m = tl.m0 + wm * C::WTM + mi * 16 + 4 * (lane >> 4);
        if (nn >= g.N) continue;
        const f32x4 v = acc[mi][ni];
        float* dst = C0 + (int64_t)nn * ldc + m;
        if (m + 3 < g.M) {
          *(float4*)dst = make_float4(v[0], v[1], v[2], v[3]);
          sqa += sq4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (m + u < g.M) {
              dst[u] = v[u];
              sqa += (double)v[u] * v[u];
            }
        }
      }
  }
#pragma unroll
  for (int h = 0; h < NBANDS; ++h) {
    if (direct) break;
    if (wm == h / BPW) {
      const int mi0 = (h % BPW) * (BR / 16);
#pragma unroll
      for (int mi = 0; mi < BR / 16; ++mi)
#pragma unroll
        for (int ni = 0; ni < C::FN; ++ni)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            img[(mi * 16 + 4 * (lane >> 4) + j) * pitch + wn * C::WTN + ni * 16 + (lane & 15) +
                (shiftvec ? (e_base + j * l3) & 3 : 0)] = acc[mi0 + mi][ni][j];
    }
    __syncthreads();
    if (btrans) {
      const int q = threadIdx.x & 15;
      const int m = tl.m0 + h * BR + 4 * q;
      for (int c = threadIdx.x >> 4; c < C::BN; c += C::NT / 16) {
        const int nn = tl.n0 + c;
        if (nn >= g.N || m >= g.M) continue;
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = img[(4 * q + u) * pitch + c];
        float* dst = C0 + (int64_t)nn * ldc + m;
        if (vec && m + 3 < g.M) {
          *(float4*)dst = make_float4(v[0], v[1], v[2], v[3]);
          sqa += sq4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (m + u < g.M) {
              dst[u] = v[u];
              sqa += (double)v[u] * v[u];
            }
        }
      }
      __syncthreads();
      continue;
    }
    if (h == 0 && bmode == 1) {  // shift = the tile's first row (always < M)
#pragma unroll
      for (int u = 0; u < 4; ++u) sh[u] = img[cq + u] + bb[u];
    }
    for (int r = rq; r < BR; r += RPI) {
      const int m = tl.m0 + h * BR + r;
      if (m >= g.M) break;
      if (shiftvec) {
        const int e = (e_base + r * l3) & 3;  // image position p holds column p - e
        float* rowp = C0 + (int64_t)m * ldc + tl.n0 - e;  // rowp + p: 16-B aligned for p % 4 == 0
        const float4 w = *(const float4*)(img + r * pitch + cq);
        const int c0 = cq - e;
        if (c0 >= 0 && tl.n0 + c0 + 3 < g.N) {
          *(float4*)(rowp + cq) = w;
          sqa += sq4(w.x, w.y, w.z, w.w);
        } else {
          const float wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (c0 + u >= 0 && tl.n0 + c0 + u < g.N) {
              rowp[cq + u] = wv[u];
              sqa += (double)wv[u] * wv[u];
            }
        }
        if (cq == 0 && e > 0) {  // the end chunk: positions BN .. BN + e - 1
          const float4 t = *(const float4*)(img + r * pitch + C::BN);
          const float tv[4] = {t.x, t.y, t.z, t.w};
          for (int u = 0; u < e; ++u)
            if (tl.n0 + C::BN - e + u < g.N) {
              rowp[C::BN + u] = tv[u];
              sqa += (double)tv[u] * tv[u];
            }
        }
        continue;
      }
      const float4 w = *(const float4*)(img + r * pitch + cq);
      const float v[4] = {w.x + bb[0], w.y + bb[1], w.z + bb[2], w.w + bb[3]};
      float* dst = (EPI != 0 || m < msplit ? Cz + (int64_t)m * ldc : C1 + (int64_t)(m - msplit) * ldc) + n;
      if (vec && n + 3 < g.N) {
        *(float4*)dst = make_float4(v[0], v[1], v[2], v[3]);
        sqa += sq4(v[0], v[1], v[2], v[3]);
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (n + u < g.N) {
            dst[u] = v[u];
            sqa += (double)v[u] * v[u];
          }
      }
      if (bmode == 1) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float dv = v[u] - sh[u];
          sa[u] += dv;
          sb[u] = fmaf(dv, dv, sb[u]);
        }
      } else if (bmode == 2) {
        const float4 y4 = *(const float4*)(bn.Y + (int64_t)m * bn.ldy + n);
        const float y[4] = {y4.x, y4.y, y4.z, y4.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float d = fmaf(y[u], balpha[u], bbeta[u]) > 0.f ? v[u] : 0.f;
          sa[u] += d;
          sb[u] = fmaf(y[u] - bmean[u], d, sb[u]);
        }
      }
    }
    __syncthreads();
  }
  if (bmode) {  // (bn mode: N % 4 == 0, one K pass, 128-row tiles -- checked on the host)
    float4* red = (float4*)smem;
    red[2 * threadIdx.x] = make_float4(sa[0], sa[1], sa[2], sa[3]);
    red[2 * threadIdx.x + 1] = make_float4(sb[0], sb[1], sb[2], sb[3]);
    __syncthreads();
    if (threadIdx.x < TPR && n < g.N) {
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), q = a;
#pragma unroll
      for (int k = 0; k < RPI; ++k) {
        const float4 x = red[2 * (threadIdx.x + k * TPR)], y = red[2 * (threadIdx.x + k * TPR) + 1];
        a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
        q.x += y.x; q.y += y.y; q.z += y.z; q.w += y.w;
      }
      const float av[4] = {a.x, a.y, a.z, a.w}, qv[4] = {q.x, q.y, q.z, q.w};
      float2* o = bn.part + (int64_t)(tl.m0 / C::BM) * bn.ldp + n;
      const float nr = (float)min(C::BM, g.M - tl.m0);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (bmode == 1) {
          const float dm = av[u] / nr;
          o[u] = make_float2(sh[u] + dm, fmaxf(fmaf(-av[u], dm, qv[u]), 0.f));
        } else {
          o[u] = make_float2(av[u], qv[u]);
        }
      }
    }
  }
  if (bn.sq) {  // (one K pass: checked on the host) fixed-order block sum, one fp64 per tile
    double* red = (double*)smem;
    const double w = wave_sum_d(sqa);
    __syncthreads();
    if (lane == 0) red[wid] = w;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
#pragma unroll
      for (int k = 0; k < C::NT / 64; ++k) t += red[k];
      bn.sq[(tl.m0 / C::BM) * (g.Np / C::BN) + tl.n0 / C::BN] = t;
    }
  }
#ifdef GM2_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  GM2_STAMP(3);
#endif
}

// ---------------------------------------------------------------------------------------------
// Epilogue 2: decoder output layer + reconstruction loss (loss_components.py:49-50 BCE(sum),
// :111-115 gene abundance) and, in training, dL/dlogit as autograd composes Sigmoid->BCE:
//   dp = (p-x)/max((1-p)p, 1e-12) + w*gamma ; dl = dp*(1-p)*p.
// (sign(colsum p) == 1 wherever p > 0, and dl == 0 wherever p == 0: no batch-wide pass needed.)
// The tile is computed TRANSPOSED: P = the output weight W9 [Gp][H] (rows = genes), Q = the last
// hidden activations A5 [Bp][H] (rows = strains), so acc holds logit^T and each lane owns FOUR
// CONSECUTIVE GENES of one strain row: 8-byte bf16 (16-byte f32) LDS image writes, one 32-bit word
// of the row-major target bits, a float4 of the bias.
// FAST (bf16 training path): hardware exp / rcp / log (~1 ulp), log(1-p) for log1p(-p), and the
// (p-x)/max(q,1e-12)*q product folded to (p-x) where q >= 1e-12 (the same value up to one
// rounding); the fp32 parity path keeps the reference's exact formula order.
// Writes dL [strain][ldd] (row-major, through an LDS image for full-line stores), zero outside the
// valid G x B box; per-tile BCE and sum(p) into loss_part[tile*2 + {0,1}]; per-(strain tile, gene)
// sums of dl into colpart (the output bias gradient).
// ---------------------------------------------------------------------------------------------
// The loss epilogue's element loop. No per-element guards: padded genes (g >= G) have a zero
// weight row and a zero bias, so their logit is exactly 0 and their BCE / sum(p) contributions are
// exact constants the kernel subtracts per tile; padded strains' sums are dropped per column. Padded dL entries are harmless: every consumer multiplies them by
// zero-padded operands (W9 shadow rows >= G, A5 rows >= B) or never reads them.
//
// FAST (bf16 training) element math, in the reference's own quantities: p = sigmoid(l) as
// rcp(1 + exp2(-l log2 e)) (hardware ~1 ulp), 1 - p formed in fp32 from p exactly as the reference
// forms it (so a p that rounds to 1.0 gives the reference's log(0) -> -100 clamp and zero gradient),
//   BCE = -max(log(x ? p : 1-p), -100)          (log(1-p) for log1p(-p): same value up to rounding)
//   dl  = (p - x) * min(p(1-p) * 1e12, 1) + w*gamma * p(1-p)
// which is the reference's ((p-x)/max(p(1-p),1e-12) + w*gamma) * (1-p) * p up to rounding. The
// selects are bit-field ops on a 0 / -1 mask from the target bit (x ? p : 1-p as |x ? p : p-1|,
// p - x as x ? p-1 : p), BCE is summed in log2 units and scaled by -ln 2 once per tile, and the
// bias arrives pre-scaled (nb = -b log2 e). BCE and sum(p) are summed per strain column and masked
// once per column (padded strains).
// Exact (fp32 parity) path: the reference's formula order, p computed first.
// (m & a) | (~m & b) as one v_bfi_b32 (the compiler rewrites the C form into compare + select)
__device__ __forceinline__ float bfi(int m, float a, float b) {
  float r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}

template <class C, typename T, bool FAST, bool WG, bool GRAD>
__device__ __forceinline__ void recon_tile(const f32x4 (&acc)[C::FM][C::FN], const uint32_t* __restrict__ xrow,
                                           int64_t ldxb, const float* bias_s, int N, int n0, int wm, int wn, int q,
                                           int c, float wgam, T* img, float& bce, float& psum,
                                           const int* xidx) {
  constexpr int PR = C::BM + 8;
  constexpr int XW = C::WTM / 32;  // target words of this wave's gene span per strain row
  static_assert(XW == 4 || XW == 2, "wave gene span");
  // strain-major order: one strain column (16 lanes x 4 genes x FM slices) at a time, so only
  // that strain's target words and one LDS row base are live (the image offsets of the FM slices
  // are immediates)
  // every strain column's target words are loaded up front (the main loop's fragment registers are
  // free now): one exposed load latency per tile instead of one per strain column
  uint32_t xwa[C::FN][XW];
#pragma unroll
  for (int ni = 0; ni < C::FN; ++ni) {
    const int sl = wn * C::WTN + ni * 16 + c;
    // (zero-copy rows: the strain's row of the resident target bits, from the tile's LDS table)
    const uint32_t* xp = xrow + (int64_t)(xidx ? xidx[sl] : n0 + sl) * ldxb;
    if (n0 + sl < N) {
      if constexpr (XW == 4) {
        const uint4 v = *(const uint4*)xp;
        xwa[ni][0] = v.x; xwa[ni][1] = v.y; xwa[ni][2] = v.z; xwa[ni][3] = v.w;
      } else {
        const uint2 v = *(const uint2*)xp;
        xwa[ni][0] = v.x; xwa[ni][1] = v.y;
      }
    } else {
#pragma unroll
      for (int k = 0; k < XW; ++k) xwa[ni][k] = 0u;
    }
  }
#pragma unroll
  for (int ni = 0; ni < C::FN; ++ni) {
    const int sl = wn * C::WTN + ni * 16 + c;  // strain (tile-local)
    const bool sok = n0 + sl < N;
    uint32_t xw[XW];
#pragma unroll
    for (int k = 0; k < XW; ++k) xw[k] = xwa[ni][k];
    // this lane's genes of word k sit at bits (mi & 1) * 16 + j after the shift by 4q
#pragma unroll
    for (int k = 0; k < XW; ++k) xw[k] >>= 4 * q;
    T* irow = img + sl * PR + wm * C::WTM + 4 * q;
    float bce_c = 0.f, ps_c = 0.f;
    f32x2_t bce2 = {0.f, 0.f}, ps2 = {0.f, 0.f};  // (FAST: pairs of elements)
    // the tile's bias slice sits in LDS (zero beyond G; pre-scaled by -log2 e on the FAST path);
    // slice mi + 1 is read while slice mi is computed
    const float* bsl = bias_s + wm * C::WTM + 4 * q;
    float4 b4n = *(const float4*)bsl;
#pragma unroll
    for (int mi = 0; mi < C::FM; ++mi) {
      const float4 b4 = b4n;
      if (mi + 1 < C::FM) b4n = *(const float4*)(bsl + (mi + 1) * 16);
      const float bn[4] = {b4.x, b4.y, b4.z, b4.w};
      float dl4[4];
      if constexpr (FAST) {
        // two elements per step in packed fp32 (v_pk_fma / v_pk_add / v_pk_mul: the register pairs
        // of the accumulator and the bias), the transcendentals, bit-field selects and clamps per
        // element; the same operations in the same order as one element at a time
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x2_t a2 = {acc[mi][ni][2 * h], acc[mi][ni][2 * h + 1]};
          const f32x2_t b2 = {bn[2 * h], bn[2 * h + 1]};
          const f32x2_t y2 = a2 * f32x2_t{-1.4426950408889634f, -1.4426950408889634f} + b2;  // -l log2 e
          const f32x2_t d2 = f32x2_t{__builtin_amdgcn_exp2f(y2.x), __builtin_amdgcn_exp2f(y2.y)} + 1.0f;
          const f32x2_t p2 = {__builtin_amdgcn_rcpf(d2.x), __builtin_amdgcn_rcpf(d2.y)};
          const f32x2_t nomp2 = p2 - 1.0f;  // -(1 - p)
          const int msk0 = __builtin_amdgcn_sbfe((int)xw[mi >> 1], (mi & 1) * 16 + 2 * h, 1);  // x ? -1 : 0
          const int msk1 = __builtin_amdgcn_sbfe((int)xw[mi >> 1], (mi & 1) * 16 + 2 * h + 1, 1);
          const float l0 = fmaxf(__builtin_amdgcn_logf(fabsf(bfi(msk0, p2.x, nomp2.x))), -144.26950408889634f);
          const float l1 = fmaxf(__builtin_amdgcn_logf(fabsf(bfi(msk1, p2.y, nomp2.y))), -144.26950408889634f);
          bce2 += f32x2_t{l0, l1};  // max(log2, -100/ln 2)
          ps2 += p2;
          const f32x2_t r2 = {bfi(msk0, nomp2.x, p2.x), bfi(msk1, nomp2.y, p2.y)};  // p - x
          // -(1 - p) p once (packed); the 1e-12 guard factor is one multiply with the clamp
          // modifier per element, and the gene-abundance term reuses the product
          const f32x2_t t2 = nomp2 * p2;
          const f32x2_t s2 = {__builtin_amdgcn_fmed3f(t2.x * -1e12f, 0.0f, 1.0f),
                              __builtin_amdgcn_fmed3f(t2.y * -1e12f, 0.0f, 1.0f)};
          f32x2_t dl2 = r2 * s2;
          if constexpr (WG) dl2 = f32x2_t{-wgam, -wgam} * t2 + dl2;
          dl4[2 * h] = dl2.x;
          dl4[2 * h + 1] = dl2.y;
        }
      } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (FAST) {
          const int msk = __builtin_amdgcn_sbfe((int)xw[mi >> 1], (mi & 1) * 16 + j, 1);  // x ? -1 : 0
          const float y = fmaf(acc[mi][ni][j], -1.4426950408889634f, bn[j]);  // -l log2 e
          const float p = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(y));
          const float nomp = p - 1.0f;  // -(1 - p)
          const float arg = bfi(msk, p, nomp);  // x ? p : p - 1
          bce_c += fmaxf(__builtin_amdgcn_logf(fabsf(arg)), -144.26950408889634f);  // max(log2, -100/ln 2)
          ps_c += p;
          const float r = bfi(msk, nomp, p);    // p - x
          const float s = __builtin_amdgcn_fmed3f(nomp * -1e12f * p, 0.0f, 1.0f);
          float dl = r * s;
          if constexpr (WG) dl = fmaf(-wgam, nomp * p, dl);
          dl4[j] = dl;
        } else {
          const uint32_t xb = xw[mi >> 1] >> ((mi & 1) * 16);
          const bool x = (xb >> j) & 1u;
          const float l = acc[mi][ni][j] + bn[j];
          const float p = 1.0f / (1.0f + expf(-l));
          bce_c += x ? -fmaxf(logf(p), -100.f) : -fmaxf(log1pf(-p), -100.f);
          ps_c += p;
          const float omp = 1.0f - p;
          const float dp = (p - (x ? 1.0f : 0.0f)) / fmaxf(omp * p, 1e-12f) + wgam;
          dl4[j] = dp * omp * p;
        }
      }
      }
      if constexpr (GRAD) {
        if constexpr (sizeof(T) == 2) {
          uint2 pk;
          pk.x = f2bf2(dl4[0], dl4[1]);
          pk.y = f2bf2(dl4[2], dl4[3]);
          *(uint2*)(irow + mi * 16) = pk;
        } else {
          *(f32x4*)(irow + mi * 16) = f32x4{dl4[0], dl4[1], dl4[2], dl4[3]};
        }
      }
    }
    if constexpr (FAST) {
      bce_c = bce2.x + bce2.y;
      ps_c = ps2.x + ps2.y;
    }
    if (sok) {
      bce += bce_c;
      psum += ps_c;
    }
  }
}

// BCE / sum(p) of one padded gene (logit exactly 0, target 0): p = 1/2, BCE = -log(1/2)
template <bool FAST>
__device__ __forceinline__ void recon_pad_const(float& e0, float& p0) {
  if constexpr (FAST) {  // the FAST element math at l = 0, x = 0
    const float p = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(0.f));
    e0 = -fmaxf(__builtin_amdgcn_logf(fabsf(p - 1.0f)), -144.26950408889634f) * 0.6931471805599453f;
    p0 = p;
  } else {
    p0 = 1.0f / (1.0f + expf(-0.f));
    e0 = -fmaxf(log1pf(-p0), -100.f);
  }
}

template <class C, typename T, bool PP, bool GRAD>
__device__ __forceinline__ void recon_loss_tile(const TileXY tl, const GemmArgs<T>& g, const float* __restrict__ bias,
                                                const uint32_t* __restrict__ xbits, int64_t ldxb,
                                                const float* __restrict__ scal, T* __restrict__ dL, int64_t ldd,
                                                float* __restrict__ loss_part, float* __restrict__ colpart,
                                                int64_t ldcol, char* smem, const int32_t* __restrict__ xrows);

// ntiles > 0: capped grid, workgroup wg takes tiles wg, wg + grid, ... (GM2_OPT_GRID_CAP bit 4)
template <class C, typename T, bool PP, bool GRAD>
__global__ __launch_bounds__(C::NT) void k_gemm_recon_loss(GemmArgs<T> g, const float* __restrict__ bias,
                                                         const uint32_t* __restrict__ xbits, int64_t ldxb,
                                                         int ntiles, const float* __restrict__ scal,
                                                         T* __restrict__ dL, int64_t ldd,
                                                         float* __restrict__ loss_part, float* __restrict__ colpart,
                                                         int64_t ldcol, const int32_t* __restrict__ xrows) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  GM2_STAMP(0);
  const int tm = g.Mp / C::BM, tn = g.Np / C::BN;
  if (ntiles == 0) {
    recon_loss_tile<C, T, PP, GRAD>(tile_of<C>(tm, tn), g, bias, xbits, ldxb, scal, dL, ldd, loss_part, colpart,
                                    ldcol, smem, xrows);
    return;
  }
  for (int t = xcd_wg(); t < ntiles; t += gridDim.x) {
    __syncthreads();
    recon_loss_tile<C, T, PP, GRAD>(tile_at<C>(t, tm, tn, 0), g, bias, xbits, ldxb, scal, dL, ldd, loss_part,
                                    colpart, ldcol, smem, xrows);
  }
}

template <class C, typename T, bool PP, bool GRAD>
__device__ __forceinline__ void recon_loss_tile(const TileXY tl, const GemmArgs<T>& g, const float* __restrict__ bias,
                                                const uint32_t* __restrict__ xbits, int64_t ldxb,
                                                const float* __restrict__ scal, T* __restrict__ dL, int64_t ldd,
                                                float* __restrict__ loss_part, float* __restrict__ colpart,
                                                int64_t ldcol, char* smem, const int32_t* __restrict__ xrows) {
  constexpr bool FAST = sizeof(T) == 2;
  // (m = genes, n = strains)
  // LDS: [0, image / staging) | per-row-group dl sums | BCE, sum(p) slots | bias slice
  constexpr int EPC = 16 / sizeof(T);
  constexpr int PR = C::BM + 8;
  constexpr int CPR = C::BM / EPC;      // 16-byte chunks per image row
  constexpr int RG = C::NT / CPR;       // row groups of the store pass
  constexpr int IMG = std::max<int>(C::LDS, C::BN * PR * (int)sizeof(T));
  float* colred = (float*)(smem + IMG);  // [RG][BM]
  float* red = colred + RG * C::BM;     // [2][32]
  float* bias_s = red + 64;             // [BM]
  int* xidx = (int*)(bias_s + C::BM);   // [BN] zero-copy strain rows of the target bits
  for (int i = threadIdx.x; i < C::BM; i += C::NT) {
    const float b = tl.m0 + i < g.M ? bias[tl.m0 + i] : 0.f;
    bias_s[i] = FAST ? b * -1.4426950408889634f : b;
  }
  if (xrows)
    for (int i = threadIdx.x; i < C::BN; i += C::NT) {
      xidx[i] = xrows[tl.n0 + i];
      GM2_DBG(xidx[i] >= 0 && (g.idx_lim == 0 || xidx[i] < g.idx_lim), kDbgReconRows);
    }
  GM2_DBG(tl.m0 + C::BM <= g.Mp && tl.n0 + C::BN <= g.Np, kDbgTile);
  f32x4 acc[C::FM][C::FN];
  if constexpr (PP)
    mainloop_pp<true, true>(g.P, g.ldp, g.Q, g.ldq, tl.m0, tl.n0, 0, g.K / E<T>::KT, smem, acc);
  else
    mainloop<C, T, true, true>(g.P, g.ldp, g.Q, g.ldq, tl.m0, tl.n0, 0, g.K / E<T>::KT, smem, acc);
  GM2_STAMP(2);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wm = wid / C::WGN, wn = wid % C::WGN;
  const int q = lane >> 4, c = lane & 15;
  const float wgam = scal[kScalWGamma];
  float bce = 0.f, psum = 0.f;
  T* img = (T*)smem;  // LDS image [BN strains][BM genes + 8] of T
  // (one element loop with the gene-abundance FMA for every preset: at w*gamma = 0 it leaves dl bit
  // for bit as it was, costs half a packed FMA per element, and keeps the kernel to one copy of the
  // loop -- with a second, FMA-free copy behind a uniform branch it spilled 42 VGPRs, with one 4)
  recon_tile<C, T, FAST, true, GRAD>(acc, xbits + ((tl.m0 + wm * C::WTM) >> 5), ldxb, bias_s, g.N, tl.n0, wm, wn, q, c,
                                     wgam, img, bce, psum, xrows ? xidx : nullptr);
  if constexpr (FAST) bce *= -0.6931471805599453f;
  GM2_STAMP(4);
  if constexpr (GRAD) {
    __syncthreads();
    // dL rows (strains) of BM genes: full 16-byte stores along each row. Thread i keeps one chunk
    // column (EPC genes) over rows i/CPR, +RG, ...: the same pass sums that chunk's dl over the
    // valid strains for the output bias gradient (the rounded values the dW9 GEMM reads).
    const int cch = threadIdx.x % CPR, r0 = threadIdx.x / CPR;
    float cs[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) cs[e] = 0.f;
    for (int r = r0; r < C::BN; r += RG) {
      const uint4 v = *(const uint4*)(img + r * PR + cch * EPC);
      // (non-temporal: the 451-MB dL stream does not displace the output-layer weights, which
      // the loss GEMM re-reads from the Infinity Cache across strain tiles)
      __builtin_nontemporal_store(u32x4_t{v.x, v.y, v.z, v.w},
                                  (u32x4_t*)(dL + (int64_t)(tl.n0 + r) * ldd + tl.m0 + cch * EPC));
      if (tl.n0 + r < g.N) {
        if constexpr (sizeof(T) == 2) {
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            cs[2 * e] += __uint_as_float(w[e] << 16);
            cs[2 * e + 1] += __uint_as_float(w[e] & 0xFFFF0000u);
          }
        } else {
          cs[0] += __uint_as_float(v.x); cs[1] += __uint_as_float(v.y);
          cs[2] += __uint_as_float(v.z); cs[3] += __uint_as_float(v.w);
        }
      }
    }
#pragma unroll
    for (int e = 0; e < EPC; ++e) colred[r0 * C::BM + cch * EPC + e] = cs[e];
  }
  bce = wave_sum(bce);
  psum = wave_sum(psum);
  if (lane == 0) { red[wid] = bce; red[32 + wid] = psum; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, b = 0.f;
    for (int w = 0; w < C::NT / 64; ++w) { a += red[w]; b += red[32 + w]; }
    // padded genes of an edge tile: logit exactly 0 -> p = 1/2, x = 0, BCE = -log(1/2) each
    // (a tile may lie wholly in the padding when Gp - G >= BM: the bf16 workspaces pad G to 256)
    const int pad_g = min(C::BM, max(0, tl.m0 + C::BM - g.M)), val_s = min(C::BN, g.N - tl.n0);
    if (pad_g > 0) {
      float e0, p0;
      recon_pad_const<FAST>(e0, p0);
      a -= (float)pad_g * (float)val_s * e0;
      b -= (float)pad_g * (float)val_s * p0;
    }
    loss_part[tl.t * 2 + 0] = a;
    loss_part[tl.t * 2 + 1] = b;
  }
  if constexpr (GRAD) {
    for (int cc = threadIdx.x; cc < C::BM; cc += C::NT) {
      const int gg = tl.m0 + cc;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < RG; ++w) v += colred[w * C::BM + cc];
      if (gg < g.M) colpart[(int64_t)(tl.n0 / C::BN) * ldcol + gg] = v;
    }
  }
#ifdef GM2_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  GM2_STAMP(3);
#endif
}

template <class C, typename T>
constexpr int recon_lds_bytes() {
  constexpr int img = std::max<int>(C::LDS, C::BN * (C::BM + 8) * (int)sizeof(T));
  constexpr int rg = C::NT / (C::BM / (16 / (int)sizeof(T)));
  return img + (rg * C::BM + 64 + C::BM + C::BN) * 4;
}

// ---------------------------------------------------------------------------------------------
// Epilogue 3: sampling / evaluation output layer. pred = sigmoid_fp32(logit) > thr: for thr = 0.5
// (the reference's extras.py:200-201 `> 0.5`) as logit > 0x33C00000, else p > thr with
// p = 1 / (1 + exp(-logit)) in fp32. The tile's predictions go through an LDS u8 image and leave as
//   * mask  u8 [m][ldm] (full-row byte runs; 16-byte stores when ldm allows), and/or
//   * bits  [m][ldb] bytes, numpy packbits(bitorder='little') rows: bit (n & 7) of byte n / 8, and/or
//   * counts int32 [m][3] += (TP, FP, FN) against the row-major target bits (metrics.py:19-64), and/or
//   * probs fp32 [m][ldpr] = p (extras.py:198).
// ---------------------------------------------------------------------------------------------
struct MaskOut {
  uint8_t* mask; int64_t ldm;
  uint8_t* bits; int64_t ldb;
  float* probs; int64_t ldpr;
  int* counts; const uint32_t* xbits; int64_t ldxb;
  float thr;
  MaskGate gate;
  MaskBand band;
};

// The certified band (MaskBand): the tile's row norms and column norms go to LDS past the staging
// ring after the main loop (mask_tile), with the tile's slot counter after them. Per element the
// epilogues add one compare (|d| <= rmax * ce + eb, MaskBand) and its wave ballot: the packed-bits
// epilogue appends a position's flagged (row, gene) pairs right there (a uniform branch, rarely
// taken); the u8 epilogue ORs the ballots and a flagged wave re-walks its fragments.
template <class C>
constexpr int band_lds_bytes() { return (C::BM + C::BN) * 4 + 16; }

// the band's per-column terms of one lane (column fragment ni): bt = b - T, ce = coef ||w_g||
// (rounded up); the rounding floor 2^-21 (|b| + T) <= 2^-21 |bt| + 2^-20 T is formed per fragment.
// Pad genes: bt = -inf, ce = -inf (never in the band)
template <class C>
struct BandCols {
  float bt[C::FN], ce[C::FN];
  __device__ __forceinline__ BandCols(const float* __restrict__ bias, const float* brn, const MaskBand& band, bool bchk,
                                      int n0, int N, int lane, int wn) {
#pragma unroll
    for (int ni = 0; ni < C::FN; ++ni) {
      const int nl = wn * C::WTN + ni * 16 + (lane & 15);
      const bool in = n0 + nl < N;
      bt[ni] = in ? bias[n0 + nl] - kMaskLogitThreshold : -INFINITY;
      ce[ni] = !in ? -INFINITY : bchk ? band.coef * brn[C::BM + nl] * (1.0f + 0x1p-20f) : 0.f;
    }
  }
  // this lane's band half-widths for row fragment mi (the largest of its four rows' norms); without
  // a band check: -1 (nothing is in it)
  __device__ __forceinline__ void widths(const float* brn, bool bchk, int r0, float (&e)[C::FN]) const {
    if (!bchk) {
#pragma unroll
      for (int ni = 0; ni < C::FN; ++ni) e[ni] = -1.f;
      return;
    }
    const float4 r4 = *(const float4*)(brn + r0);
    const float rmax = fmaxf(fmaxf(r4.x, r4.y), fmaxf(r4.z, r4.w));
#pragma unroll
    for (int ni = 0; ni < C::FN; ++ni)
      e[ni] = fmaf(rmax, ce[ni], fmaf(0x1p-21f, fabsf(bt[ni]), 0x1p-20f * kMaskLogitThreshold));
  }
};

// A band entry past its shard's capacity only sets the lane's `ovf`; after its epilogue the tile
// flags the 256 x 256 block it lies in (the first lane to flag it lists it) for k_band_tile_fix's
// whole-block fp64 recompute. (Flagging at each of the unrolled epilogue's 128 append sites had grown
// the bit-packing mask kernel from 120 to 208 KB of code and its launch from 5.0 to 5.7 ms; deferring
// every append to one rolled loop, 49 KB, measured 5.4 ms: profiles/r06_mask_code_size_ab.txt.)
__device__ __forceinline__ void band_spill_block(const MaskBand& b, int m0, int n0) {
  const unsigned blk = (unsigned)(m0 >> 8) * (unsigned)b.obn + (unsigned)(n0 >> 8);
  GM2_DBG(blk < b.oblocks && (n0 >> 8) < b.obn, kDbgBandBlock);
  if (blk >= b.oblocks) return;  // (cannot happen: tiles lie inside the block grid)
  if (atomicExch(b.oflag + blk, 1u) == 0u) b.olist[atomicAdd(b.ocount, 1u)] = blk;
}

// one wave's band elements: walk(visit) calls visit(in, row, gene) for every fragment position in a
// fixed order; per position with flagged lanes, one reservation for all of them (an LDS counter
// for the tile's slots, else the shard's counter) and each flagged lane's entry at its prefix
template <class C, class F>
__device__ __forceinline__ void band_walk(const MaskBand& b, int tile, char* smem, int lane, bool& ovf, F&& walk) {
  unsigned* lcount = (unsigned*)(smem + C::LDS) + C::BM + C::BN;
  const int sh = blockIdx.x % kBandShards;
  uint2* shard = b.list + (size_t)sh * b.cap;
  walk([&](bool in, int r, int gcol) {
    const uint64_t bal = __ballot(in);
    if (!bal) return;
    const unsigned pre = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
    unsigned base = 0;
    if (lane == 0) base = atomicAdd(b.tslots ? lcount : b.counts + sh, (unsigned)__popcll(bal));
    const unsigned i = __shfl(base, 0, 64) + pre;
    if (!in) return;
    const uint2 e = make_uint2((unsigned)r, (unsigned)gcol);
    if (!b.tslots) {
      if (i < b.cap) shard[i] = e;
      else ovf = true;
    } else if (i < (unsigned)b.tslots) {
      b.tlist[(size_t)tile * b.tslots + i] = e;
    } else if (!b.drop_overflow) {  // past the tile's slots: the shard (rare)
      const unsigned k = atomicAdd(b.counts + sh, 1u);
      if (k < b.cap) shard[k] = e;
      else ovf = true;
    }
  });
}
// one fragment position's band elements (bal = the wave's ballot of `in`; wave-uniform call): one
// reservation for all of them, as band_walk's visitor
template <class C>
__device__ __forceinline__ void band_add(const MaskBand& b, int tile, char* smem, int lane, uint64_t bal, bool in,
                                         int r, int gcol, bool& ovf) {
  unsigned* lcount = (unsigned*)(smem + C::LDS) + C::BM + C::BN;
  const int sh = blockIdx.x % kBandShards;
  const unsigned pre = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
  unsigned base = 0;
  if (lane == 0) base = atomicAdd(b.tslots ? lcount : b.counts + sh, (unsigned)__popcll(bal));
  const unsigned i = __shfl(base, 0, 64) + pre;
  if (!in) return;
  const uint2 e = make_uint2((unsigned)r, (unsigned)gcol);
  uint2* shard = b.list + (size_t)sh * b.cap;
  if (!b.tslots) {
    if (i < b.cap) shard[i] = e;
    else ovf = true;
  } else if (i < (unsigned)b.tslots) {
    b.tlist[(size_t)tile * b.tslots + i] = e;
  } else if (!b.drop_overflow) {
    const unsigned k = atomicAdd(b.counts + sh, 1u);
    if (k < b.cap) shard[k] = e;
    else ovf = true;
  }
}

// after the epilogue's barrier: the tile's slot count
template <class C>
__device__ __forceinline__ void band_close(const MaskBand& b, int tile, char* smem) {
  if (!b.tslots || threadIdx.x != 0) return;
  const unsigned n = ((const unsigned*)(smem + C::LDS))[C::BM + C::BN];
  b.tcount[tile] = n;
  if (b.drop_overflow && n > (unsigned)b.tslots) return;  // (re-run by the split kernel, counted there)
  if (n) atomicAdd(b.tfound + blockIdx.x % kBandShards, min(n, (unsigned)b.tslots));
  if (b.tiles_done) atomicAdd(b.tiles_done + blockIdx.x % kSplitShards, 1u);
}

template <class C, typename T, bool PP, bool BITS, bool S3>
__device__ __forceinline__ void mask_tile(const TileXY tl, const GemmArgs<T>& g, const float* __restrict__ bias,
                                          const MaskOut& o, char* smem);

// PP: the 256x256 bf16 ping-pong main loop in its S3 form (the bf16x3 sampling decode: hi.hi +
// hi.lo + lo.hi over operands split by launch_split3, K' = 2H, decode_split3). LOOP (gated 128 x
// 128 launches, usually the complement of the split kernel with few tiles to run): a grid of a few
// workgroups per CU loops over the tiles t, t + grid, ... instead of one workgroup per tile.
template <class C, typename T, bool PP = false, bool BITS = false, bool LOOP = false, bool S3 = true>
__global__ __launch_bounds__(C::NT) void k_gemm_mask(GemmArgs<T> g, const float* __restrict__ bias, MaskOut o) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tm = g.Mp / C::BM, tn = g.Np / C::BN, ntile = tm * tn;
  if constexpr (!LOOP) {
    const TileXY tl = tile_of<C>(tm, tn);
    if (o.gate.run) {  // the verdict of the tile's 256 x 256 block (uniform per workgroup)
      if (tile_level(o.gate, tl.m0, tl.n0) != o.gate.run) return;  // (tcount: zeroed by the caller)
      if (threadIdx.x == 0) atomicAdd(o.gate.tiles + blockIdx.x % kSplitShards, 1u);
    }
    mask_tile<C, T, PP, BITS, S3>(tl, g, bias, o, smem);
  } else {
    static_assert(!PP && !BITS, "tile loop: the 128 x 128 kernel");
    // the workgroup's tiles t0 + k G: their gate verdicts NT at a time, in parallel (one ballot word
    // per wave in LDS past the band region), then the runnable ones in order
    const int G = gridDim.x, t0 = xcd_wg(), lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t* vm = (uint64_t*)(smem + C::LDS + band_lds_bytes<C>());
    for (int kb = 0; t0 + kb * G < ntile; kb += C::NT) {
      __syncthreads();  // (the previous pass's words are read)
      const int t = t0 + (kb + (int)threadIdx.x) * G;
      bool run = false;
      if (t < ntile) {
        const TileXY tl = tile_at<C>(t, tm, tn, 0);
        run = !o.gate.run || tile_level(o.gate, tl.m0, tl.n0) == o.gate.run;
      }
      const uint64_t bw = __ballot(run);
      if (lane == 0) vm[wid] = bw;
      __syncthreads();
      unsigned nrun = 0;
#pragma unroll 1
      for (int w = 0; w < C::NT / 64; ++w) {
        const uint64_t v = vm[w];
        uint64_t m = ((uint64_t)__builtin_amdgcn_readfirstlane((unsigned)(v >> 32)) << 32) |
                     __builtin_amdgcn_readfirstlane((unsigned)v);
        while (m) {
          const int i = __builtin_ctzll(m);
          m &= m - 1;
          ++nrun;
          __syncthreads();  // (the previous tile's epilogue is done with LDS)
          mask_tile<C, T, PP, BITS, S3>(tile_at<C>(t0 + (kb + w * 64 + i) * G, tm, tn, 0), g, bias, o, smem);
        }
      }
      if (o.gate.run && nrun && threadIdx.x == 0) atomicAdd(o.gate.tiles + blockIdx.x % kSplitShards, nrun);
    }
  }
}

// The tiered output layer (GM2_OPT_SAMPLE_SINGLE): one 256x256 workgroup per tile takes its block's
// verdict -- exact tiles return at once (the exact kernel's), single-product tiles run one bf16
// product over the rounded operands (o1: K = H, the wide band, overflow dropped) and, when their band
// overflowed its slots, the same tile again as bf16x3 (o3) in place; split tiles run bf16x3 alone.
// One launch for both bf16 tiers: no second grid of workgroups that mostly exit.
template <class C, typename T, bool BITS>
__global__ __launch_bounds__(C::NT) void k_gemm_mask_tiered(GemmArgs<T> g1, GemmArgs<T> g3,
                                                            const float* __restrict__ bias, MaskOut o1, MaskOut o3) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const TileXY tl = tile_of<C>(g3.Mp / C::BM, g3.Np / C::BN);
  const int lv = tile_level(o3.gate, tl.m0, tl.n0);
  if (lv == 2) return;
  if (lv == 3) {
    mask_tile<C, T, true, BITS, false>(tl, g1, bias, o1, smem);
    __syncthreads();  // (band_close's count in LDS, read by every thread)
    if (((const unsigned*)(smem + C::LDS))[C::BM + C::BN] <= (unsigned)o1.band.tslots) return;  // (counted)
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicAdd(o3.gate.tiles + blockIdx.x % kSplitShards, 1u);
  mask_tile<C, T, true, BITS, true>(tl, g3, bias, o3, smem);
}

template <class C, typename T, bool PP, bool BITS, bool S3>
__device__ __forceinline__ void mask_tile(const TileXY tl, const GemmArgs<T>& g, const float* __restrict__ bias,
                                          const MaskOut& o, char* smem) {
  const bool bchk = o.band.rn != nullptr;
  // the tile's row and column norms (one per thread: NT = BM + BN), loaded before the main loop and
  // staged to LDS after it (its first counted wait covers the load; no stall in front of the loop)
  static_assert(C::NT == C::BM + C::BN, "one norm per thread");
  float nrm = 0.f;
  if (bchk) nrm = threadIdx.x < C::BM ? o.band.rn[tl.m0 + threadIdx.x] : o.band.cn[tl.n0 + threadIdx.x - C::BM];
  const float* brn = (const float*)(smem + C::LDS);  // [BM] row norms, then [BN] column norms
  f32x4 acc[C::FM][C::FN];
  if constexpr (PP) {
    static_assert(std::is_same_v<C, Big> && sizeof(T) == 2, "ping-pong: 256x256 bf16");
    // (S3: the split's K' = 2H form; else one product over K = H, the single-product tier)
    mainloop_pp<true, true, 0, S3>(g.P, g.ldp, g.Q, g.ldq, tl.m0, tl.n0, 0, g.K / E<T>::KT, smem, acc);
  } else {
    mainloop<C, T, true, true>(g.P, g.ldp, g.Q, g.ldq, tl.m0, tl.n0, 0, g.K / E<T>::KT, smem, acc);
  }
  if (bchk) {
    ((float*)(smem + C::LDS))[threadIdx.x] = nrm;
    if (threadIdx.x == 0) ((unsigned*)(smem + C::LDS))[C::BM + C::BN] = 0u;
    __syncthreads();
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wm = wid / C::WGN, wn = wid % C::WGN;
  const BandCols<C> bc(bias, brn, o.band, bchk, tl.n0, g.N, lane, wn);
  uint64_t bandw = 0;  // this wave's band flags, OR-ed over its fragment positions
  bool ovf = false;    // an entry of this lane's found its shard full (band_spill_block)
  if constexpr (BITS) {
    static_assert(PP, "bit-image epilogue: the split decode's kernel");
    {
      // packed bits straight from the fragments: lane l of a 16x16 fragment holds row 4(l>>4) + j,
      // column l&15, so one ballot per (mi, ni, j) yields 16 gene bits for each of 4 rows; lane r < 4
      // gathers row r's 64 bits over the wave's 4 column fragments and writes them to a [BM][32 B]
      // bit image (one ds_write_b64 per (mi, j), where the u8 image took one byte store per logit).
      // The bit is d = acc + (b - T) > 0 (pad genes: d = -inf); d and acc + b round differently
      // only inside the band, which the recompute decides.
      const int sh = 16 * (lane & 3);
#pragma unroll
      for (int mi = 0; mi < C::FM; ++mi) {
        float e[C::FN];
        bc.widths(brn, bchk, wm * C::WTM + mi * 16 + 4 * (lane >> 4), e);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uint64_t rb = 0;
          const int r = tl.m0 + wm * C::WTM + mi * 16 + 4 * (lane >> 4) + j;
          const bool rok = r < g.M;
#pragma unroll
          for (int ni = 0; ni < C::FN; ++ni) {
            const float d = acc[mi][ni][j] + bc.bt[ni];
            const uint64_t bal = __ballot(d > 0.f);
            rb |= ((bal >> sh) & 0xFFFFull) << (16 * ni);
            // the band elements of this position appended at once (a uniform branch, rarely taken)
            const bool inb = fabsf(d) <= e[ni] && rok;
            const uint64_t bb = __ballot(inb);
            if (bb) band_add<C>(o.band, tl.t, smem, lane, bb, inb, r, tl.n0 + wn * C::WTN + ni * 16 + (lane & 15), ovf);
          }
          if (lane < 4)
            *(uint64_t*)(smem + (wm * C::WTM + mi * 16 + 4 * lane + j) * (C::BN / 8) + wn * (C::WTN / 8)) = rb;
          __builtin_amdgcn_sched_barrier(0);  // (one row quad at a time: the ballots' SGPR pairs stay few)
        }
      }
      if (ovf) band_spill_block(o.band, tl.m0, tl.n0);
      __syncthreads();
      band_close<C>(o.band, tl.t, smem);
      constexpr int BPR = C::BN / 8;
      const int rows = min(C::BM, g.M - tl.m0);
      if (o.bits) {
        for (int i = threadIdx.x; i < rows * (BPR / 16); i += C::NT) {
          const int r = i / (BPR / 16), cc = i % (BPR / 16);
          if (tl.n0 / 8 + cc * 16 >= o.ldb) continue;  // (pad genes past the row pitch: all zero)
          *(uint4*)(o.bits + (int64_t)(tl.m0 + r) * o.ldb + tl.n0 / 8 + cc * 16) = *(const uint4*)(smem + r * BPR + cc * 16);
        }
      }
      if (o.mask) {
        // u8 masks expanded from the bit image (gm2_decode_mask): one lane per 4-B aligned dword of a
        // row's 256-byte segment, so a wave instruction writes one row's bytes contiguously at any row
        // alignment (the rows of a [n][G] mask are not 16-B aligned at odd G; the byte image's write-out
        // took one byte store per element there); the partial dwords at the segment's two ends and at
        // the gene edge by bytes (the neighbouring tiles own the rest of those dwords)
        static_assert(BPR == 32, "eight bit words per tile row");
        const int cols = min(C::BN, g.N - tl.n0);
        for (int r = wid; r < rows; r += C::NT / 64) {
          uint8_t* row = o.mask + (int64_t)(tl.m0 + r) * o.ldm + tl.n0;
          const int a = (int)((uintptr_t)row & 3);
          const uint32_t* bw = (const uint32_t*)(smem + r * BPR);
          for (int k = lane; k < 64 + (a != 0); k += 64) {
            const int c0 = 4 * k - a;  // tile column of the dword's first byte (-a at k = 0)
            uint32_t x;                // its four mask bits
            if (c0 < 0) {
              x = (bw[0] << a) & 0xFu;
            } else {
              const int q = c0 >> 5;
              const uint64_t w = (uint64_t)bw[q] | ((uint64_t)(q + 1 < 8 ? bw[q + 1] : 0u) << 32);
              x = (uint32_t)(w >> (c0 & 31)) & 0xFu;
            }
            if (c0 >= 0 && c0 + 3 < cols) {
              *(uint32_t*)(row + c0) = (x * 0x00204081u) & 0x01010101u;  // (row - a + 4k: aligned)
            } else {
#pragma unroll
              for (int t = 0; t < 4; ++t)
                if (c0 + t >= 0 && c0 + t < cols) row[c0 + t] = (uint8_t)((x >> t) & 1u);
            }
          }
        }
      }
      return;
    }
  }
  constexpr int PI = C::BN + 16;  // u8 image pitch
  uint8_t* img = (uint8_t*)smem;  // [BM][PI] (mainloop staging is free after its last barrier)
  const bool half = o.thr == 0.5f;
#pragma unroll
  for (int mi = 0; mi < C::FM; ++mi) {
    float e[C::FN];
    bc.widths(brn, bchk, wm * C::WTM + mi * 16 + 4 * (lane >> 4), e);
#pragma unroll
    for (int ni = 0; ni < C::FN; ++ni) {
      const int nl = wn * C::WTN + ni * 16 + (lane & 15);
      const int n = tl.n0 + nl;
      const float bnv = n < g.N ? bias[n] : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ml = wm * C::WTM + mi * 16 + 4 * (lane >> 4) + j;
        const int m = tl.m0 + ml;
        const float l = acc[mi][ni][j] + bnv;
        float p = 0.f;
        if (o.probs || !half) p = 1.0f / (1.0f + expf(-l));
        const bool pred = n < g.N && (half ? l > kMaskLogitThreshold : p > o.thr);
        img[ml * PI + nl] = pred ? 1 : 0;
        if (o.probs && m < g.M && n < g.N) o.probs[(int64_t)m * o.ldpr + n] = p;
        if (bchk) bandw |= __ballot(fabsf(acc[mi][ni][j] + bc.bt[ni]) <= e[ni]);
      }
    }
  }
  if (bandw) {  // append this wave's band elements (unrolled: acc stays in registers)
    band_walk<C>(o.band, tl.t, smem, lane, ovf, [&](auto&& visit) {
#pragma unroll
      for (int mi = 0; mi < C::FM; ++mi) {
        float e[C::FN];
        bc.widths(brn, bchk, wm * C::WTM + mi * 16 + 4 * (lane >> 4), e);
#pragma unroll
        for (int ni = 0; ni < C::FN; ++ni)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int ml = wm * C::WTM + mi * 16 + 4 * (lane >> 4) + j;
            visit(fabsf(acc[mi][ni][j] + bc.bt[ni]) <= e[ni] && tl.m0 + ml < g.M, tl.m0 + ml,
                  tl.n0 + wn * C::WTN + ni * 16 + (lane & 15));
          }
      }
    });
  }
  if (ovf) band_spill_block(o.band, tl.m0, tl.n0);
  __syncthreads();
  band_close<C>(o.band, tl.t, smem);
  const int rows = min(C::BM, g.M - tl.m0);
  if (o.mask) {
    // one row per 8 threads' 16-byte pieces (or byte runs when the rows are not 16-B aligned)
    const bool vec = (o.ldm & 15) == 0 && (((uintptr_t)o.mask) & 15) == 0 && tl.n0 + C::BN <= g.N;
    if (vec) {
      constexpr int CPR = C::BN / 16;
      for (int i = threadIdx.x; i < rows * CPR; i += C::NT) {
        const int r = i / CPR, cc = i % CPR;
        *(uint4*)(o.mask + (int64_t)(tl.m0 + r) * o.ldm + tl.n0 + cc * 16) = *(const uint4*)(img + r * PI + cc * 16);
      }
    } else {
      const int cols = min(C::BN, g.N - tl.n0);
      for (int i = threadIdx.x; i < rows * C::BN; i += C::NT) {
        const int r = i / C::BN, cc = i % C::BN;
        if (cc < cols) o.mask[(int64_t)(tl.m0 + r) * o.ldm + tl.n0 + cc] = img[r * PI + cc];
      }
    }
  }
  if (o.bits) {
    // 8 image bytes -> one packed byte; BN / 8 bytes per row, written 16 at a time
    constexpr int BPR = C::BN / 8;
    static_assert(BPR % 16 == 0, "packed row piece");
    for (int i = threadIdx.x; i < rows * (BPR / 16); i += C::NT) {
      const int r = i / (BPR / 16), cc = i % (BPR / 16);
      if (tl.n0 / 8 + cc * 16 >= o.ldb) continue;  // (pad genes past the row pitch: all zero)
      uint32_t w[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const uint2 e = *(const uint2*)(img + r * PI + cc * 128 + (k * 4 + b) * 8);
          const uint32_t lo = e.x * 0x10204080u, hi = e.y * 0x10204080u;  // gather byte LSBs
          v |= (((lo >> 28) | ((hi >> 28) << 4)) & 0xFFu) << (8 * b);
        }
        w[k] = v;
      }
      *(uint4*)(o.bits + (int64_t)(tl.m0 + r) * o.ldb + tl.n0 / 8 + cc * 16) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
  if (o.counts) {
    // per-row TP / FP / FN of this tile against the target bits; integer atomics (exact)
    constexpr int WPR = C::BN / 32;  // target words per tile row
    for (int i = threadIdx.x; i < rows * WPR; i += C::NT) {
      const int r = i / WPR, k = i % WPR;
      uint32_t pw = 0;
#pragma unroll
      for (int b = 0; b < 32; ++b) pw |= (uint32_t)img[r * PI + k * 32 + b] << b;
      const uint32_t xw = o.xbits[(int64_t)(tl.m0 + r) * o.ldxb + (tl.n0 >> 5) + k];
      int* cr = o.counts + (int64_t)(tl.m0 + r) * 3;
      const int tp = __builtin_popcount(pw & xw), fp = __builtin_popcount(pw & ~xw), fn = __builtin_popcount(~pw & xw);
      if (tp) atomicAdd(cr + 0, tp);
      if (fp) atomicAdd(cr + 1, fp);
      if (fn) atomicAdd(cr + 2, fn);
    }
  }
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// live timing of one kernel class (bench.py's roofline leg): event pairs on the launch stream
// ------------------------------------------------------------------------------------------------
namespace {
struct TimingState {
  int classes = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  std::vector<int> cls;  // the class of each used event pair
  size_t used = 0;
  std::map<int, std::pair<double, int64_t>> last;  // per-class totals of the last timed region
};
TimingState& tstate() {
  static TimingState t;
  return t;
}
}  // namespace

void timing_begin(int classes) {
  TimingState& t = tstate();
  t.classes = classes;
  t.used = 0;
}

void timing_end(double* total_ms, int64_t* launches) {
  TimingState& t = tstate();
  double tot = 0.0;
  t.last.clear();
  for (size_t i = 0; i < t.used; ++i) {
    hipError_t e = hipEventSynchronize(t.ev[i].second);
    if (e != hipSuccess) throw Gm2Error("timing: %s", hipGetErrorString(e));
    float ms = 0.f;
    e = hipEventElapsedTime(&ms, t.ev[i].first, t.ev[i].second);
    if (e != hipSuccess) throw Gm2Error("timing: %s", hipGetErrorString(e));
    tot += ms;
    auto& l = t.last[t.cls[i]];
    l.first += ms;
    l.second += 1;
  }
  *total_ms = tot;
  *launches = (int64_t)t.used;
  t.classes = 0;
  t.used = 0;
}

void timing_class(int cls, double* total_ms, int64_t* launches) {
  const TimingState& t = tstate();
  auto it = t.last.find(cls);
  *total_ms = it == t.last.end() ? 0.0 : it->second.first;
  *launches = it == t.last.end() ? 0 : it->second.second;
}

TimedLaunch::TimedLaunch(int c, hipStream_t st) : idx(-1), s(st), cls(c) {
  TimingState& t = tstate();
  if (!(t.classes & cls)) return;
  if (t.used == t.ev.size()) {
    hipEvent_t a, b;
    // (device-scope release: no L2 write-back around the timed kernel)
    if (hipEventCreateWithFlags(&a, hipEventReleaseToDevice) != hipSuccess ||
        hipEventCreateWithFlags(&b, hipEventReleaseToDevice) != hipSuccess)
      throw Gm2Error("hipEventCreate");
    t.ev.push_back({a, b});
  }
  idx = (int)t.used++;
  if (t.cls.size() < t.used) t.cls.resize(t.used);
  t.cls[idx] = cls;
  if (hipEventRecord(t.ev[idx].first, s) != hipSuccess) throw Gm2Error("hipEventRecord");
}

TimedLaunch::~TimedLaunch() {
  if (idx >= 0) (void)hipEventRecord(tstate().ev[idx].second, s);
}

// ------------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------------
template <typename T>
static void check_gemm(const GemmArgs<T>& g, int tile) {
  if (g.K % kKPad || g.Mp % tile || g.Np % tile || g.M > g.Mp || g.N > g.Np || g.M <= 0 || g.N <= 0)
    throw Gm2Error("gemm: bad dims M=%d N=%d K=%d Mp=%d Np=%d (tile %d)", g.M, g.N, g.K, g.Mp, g.Np, tile);
  if ((g.pk ? g.ldp < g.K : g.ldp < g.Mp) || (g.qk ? g.ldq < g.K : g.ldq < g.Np)) throw Gm2Error("gemm: ld too small");
  if (((uintptr_t)g.P | (uintptr_t)g.Q) & 15) throw Gm2Error("gemm: operands not 16-B aligned");
  if ((g.ldp * sizeof(T)) % 16 || (g.ldq * sizeof(T)) % 16) throw Gm2Error("gemm: ld not 16-B multiple");
}

// Tile / split-K plan. Big tiles when they alone fill the chip, or when K is long enough that a
// split-K slab round trip is cheap next to the work; otherwise the 128-tile, split only when it
// leaves most CUs idle (and never below 8 K-steps per slice).
// (split-K factor for the 128-tile GEMMs that alone fill the chip with one short-K tile per CU, the
// hidden-layer GEMMs: 256 tiles, 16 K-steps: opts().small_split > 1 puts that many tiles on each
// CU so one's loads hide behind another's MFMAs; default 1)

template <typename T>
GemmPlan plan_gemm(const GemmArgs<T>& g) {
  const int nk = g.K / E<T>::KT;
  // (the exact-fp32 path stays on the 128x128 tiles: its K-step partial sums double the accumulator
  // registers, which the 256x256 tile's 8 waves cannot hold)
  const int tiles_big = (sizeof(T) == 2 && g.Mp % 256 == 0 && g.Np % 256 == 0) ? (g.Mp / 256) * (g.Np / 256) : 0;
  const int tiles_small = (g.Mp / 128) * (g.Np / 128);
  // (up to 32 K-slices: a launch with a few tiles -- the small-batch plans, e.g. the input layer and
  // the output layer's input gradient at batch 32 / 64: 8 tiles of 128 x 128 over K = 55,040 --
  // fills the chip; at most 8 had left 192 CUs idle, 117 -> ~30 us each at batch 64; the split
  // slabs are summed in slice order by their consumers, deterministic)
  auto cap = [&](int s) { return std::max(1, std::min({s, 32, std::max(1, nk / 8)})); };
  if (tiles_big >= 256) return {256, 1};
  if (tiles_big > 0 && g.K >= 8192) return {256, cap((256 + tiles_big - 1) / tiles_big)};
  if (tiles_small >= 192) {
    const int ss = opts().small_split;
    return {128, (ss > 1 && tiles_small < 1024 && nk >= 8) ? cap(ss) : 1};
  }
  return {128, cap((256 + tiles_small - 1) / tiles_small)};
}

template <typename T>
static bool use_big(const GemmArgs<T>& g) {
  return plan_gemm(g).tile == 256;
}

// Main-loop selection for the 256x256 bf16 tiles: the ping-pong loop (default; measured
// +15-20 % on the long-K GEMMs of the v0 step, profiles/r02_gemm_bench.txt) or the two-stage loop
// (option GM2_OPT_GEMM_PP = 0, or env GM2_GEMM_PP=0 for the process defaults); both parity-tested.
static bool pp_enabled() { return opts().gemm_pp != 0; }

// waves per block (GM2_OPT_SMALL_WAVES: 4 or 8; 8: step 3.52 -> 3.46 ms, profiles/r02_ab_small_waves.txt)
// and LDS ring depth (GM2_OPT_SMALL_STAGES: 4 or 5) of the 128x128 fp32-store GEMM tiles

// call f(Cfg{}) with the 128x128 fp32-store tile configuration the options select
// (round 6 measured a 4-wave, 2-stage form with two workgroups per CU -- GM2_OPT_SMALL_PAIR, commits
// a952803 / 09afbbc -- neutral to slower at step level and removed it: profiles/r06_small_pair_ab.txt)
template <typename T, class F>
static auto small_cfg(F&& f) {
  return opts().small_waves == 8 ? f(SmallDeep8{}) : f(SmallDeep{});
}

// GM2_OPT_GRID_CAP bits: 1 = the output-layer weight-gradient GEMM (side stream, beside the
// hidden-layer backward chain), 2 = the input-layer one (beside the side stream's last hidden-layer
// weight gradients) on a capped grid -- same rounds, the last round's idle CUs free for the rest
// (default 2, dWe0 only: -18 us/step; bit 1 (dW9) measured 20-40 us/step slower: the chain's
// 256-tile GEMMs get 41 CUs (6 rounds) while dW9 runs, profiles/r02_grid_cap_ab_*)
static int grid_cap_bits() { return opts().grid_cap; }

// hipFuncAttributeMaxDynamicSharedMemorySize is per device: remember (device, kernel) pairs
static void ensure_lds_attr(const void* fn, int bytes) {
  static std::mutex mu;
  static std::set<std::pair<int, const void*>> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) throw Gm2Error("hipGetDevice");
  std::lock_guard<std::mutex> lk(mu);
  if (done.count({dev, fn})) return;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess)
    throw Gm2Error("hipFuncSetAttribute(MaxDynamicSharedMemorySize=%d)", bytes);
  done.insert({dev, fn});
}

// compute units of the current device (cached per device)
static int device_cus() {
  static std::mutex mu;
  static std::map<int, int> cus;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) throw Gm2Error("hipGetDevice");
  std::lock_guard<std::mutex> lk(mu);
  auto it = cus.find(dev);
  if (it != cus.end()) return it->second;
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    throw Gm2Error("hipDeviceGetAttribute(MultiprocessorCount)");
  return cus[dev] = std::max(n, 1);
}

template <class C, typename T, bool AK, bool BK, bool PP, int IDX = 0, int EPI = 0>
static void store_launch_k(const GemmArgs<T>& a, int tiles, float* C0, float* C1, int msplit, int64_t ldc, int64_t slab,
                           const float* bias, const StoreEpi& bn, hipStream_t s) {
  // (zero-copy rows: the index table after the staging ring -- a tile's rows, or a split's k-rows)
  constexpr int table_max = IDX == 1 ? C::BM * 4 : IDX == 2 ? kMaxIdxRows * 4 : 0;
  static_assert(C::LDS + table_max <= 160 * 1024, "LDS budget");
  const int lds = C::LDS + (IDX == 1 ? C::BM * 4 : IDX == 2 ? a.k_per_split * 4 : 0);
  if (lds > 160 * 1024) throw Gm2Error("gemm: %d bytes of LDS", lds);
  if (IDX == 2 && a.k_per_split > kMaxIdxRows) throw Gm2Error("zero-copy rows: %d k-rows per split", a.k_per_split);
  ensure_lds_attr((const void*)k_gemm_store<C, T, AK, BK, PP, IDX, EPI>, C::LDS + table_max);
  int grid = tiles;
  StoreEpi ep = bn;
  if (bn.ntiles) {  // capped grid: the same number of rounds on fewer CUs
    const int cus = device_cus(), rounds = (tiles + cus - 1) / cus;
    grid = (tiles + rounds - 1) / rounds;
    ep.ntiles = grid < tiles ? tiles : 0;
  }
  hipLaunchKernelGGL((k_gemm_store<C, T, AK, BK, PP, IDX, EPI>), dim3(grid), dim3(C::NT), lds, s, a, C0, C1 ? C1 : C0,
                     C1 ? msplit : (1 << 30), ldc, slab, bias, ep);
}

// the specialised epilogue a 256x256 launch can take (k_gemm_store EPI): 1 = plain fp32 store,
// 2 = transposed straight from the accumulators (env GM2_TRANS_DIRECT=1, A/B), 3 = transposed
// through LDS, 0 = general
static int store_epi(const GemmArgs<bf16_t>& a, float* C0, float* C1, int msplit, int64_t ldc, int64_t slab,
                     const float* bias, const StoreEpi& bn) {
  static const bool trans_direct = [] {
    const char* e = std::getenv("GM2_TRANS_DIRECT");
    return e && e[0] == '1';
  }();
  const bool aligned = ((ldc | slab) & 3) == 0 && (((uintptr_t)C0) & 15) == 0;
  if (bias || bn.mode || (C1 && msplit < a.M)) return 0;
  if (bn.trans) return aligned ? (trans_direct ? 2 : 3) : 0;
  return 1;
}

template <class C, typename T, bool AK, bool BK, bool PP, int IDX>
static void store_launch_epi(const GemmArgs<T>& a, int tiles, float* C0, float* C1, int msplit, int64_t ldc,
                             int64_t slab, const float* bias, const StoreEpi& bn, hipStream_t s) {
  switch (store_epi(a, C0, C1, msplit, ldc, slab, bias, bn)) {
    case 1: return store_launch_k<C, T, AK, BK, PP, IDX, 1>(a, tiles, C0, C1, msplit, ldc, slab, bias, bn, s);
    case 2: return store_launch_k<C, T, AK, BK, PP, IDX, 2>(a, tiles, C0, C1, msplit, ldc, slab, bias, bn, s);
    case 3: return store_launch_k<C, T, AK, BK, PP, IDX, 3>(a, tiles, C0, C1, msplit, ldc, slab, bias, bn, s);
    default: return store_launch_k<C, T, AK, BK, PP, IDX, 0>(a, tiles, C0, C1, msplit, ldc, slab, bias, bn, s);
  }
}

template <class C, typename T, bool AK, bool BK>
static void store_launch(const GemmArgs<T>& a, int tiles, float* C0, float* C1, int msplit, int64_t ldc, int64_t slab,
                         const float* bias, const StoreEpi& bn, hipStream_t s) {
  if constexpr (std::is_same_v<C, Big> && sizeof(T) == 2) {
    if (a.prow || a.qrow) {  // zero-copy rows: the input layer's two GEMMs (gemm_idx_ok checked)
      if (!pp_enabled()) throw Gm2Error("zero-copy rows need the ping-pong main loop");
      if constexpr (AK && BK) {
        if (a.prow && !a.qrow) return store_launch_epi<C, T, AK, BK, true, 1>(a, tiles, C0, C1, msplit, ldc, slab, bias, bn, s);
      }
      if constexpr (AK && !BK) {
        if (a.qrow && !a.prow) return store_launch_epi<C, T, AK, BK, true, 2>(a, tiles, C0, C1, msplit, ldc, slab, bias, bn, s);
      }
      throw Gm2Error("zero-copy rows: layout not instantiated");
    }
    if (pp_enabled()) return store_launch_epi<C, T, AK, BK, true, 0>(a, tiles, C0, C1, msplit, ldc, slab, bias, bn, s);
  }
  if (a.prow || a.qrow) throw Gm2Error("zero-copy rows: bf16 256x256 tiles only");
  store_launch_k<C, T, AK, BK, false>(a, tiles, C0, C1, msplit, ldc, slab, bias, bn, s);
}

template <class C, typename T>
static int store_impl(const GemmArgs<T>& g, int splits, float* C0, float* C1, int msplit, int64_t ldc, int64_t slab,
                      const float* bias, const StoreEpi& bn, hipStream_t s) {
  GemmArgs<T> a = g;
  const int kt = E<T>::KT;
  const int nkt = g.K / kt;
  splits = std::max(1, std::min(splits, nkt));
  a.k_per_split = (int)(round_up(nkt, splits) / splits) * kt;
  splits = (int)((g.K + a.k_per_split - 1) / a.k_per_split);
  const int tiles = (g.Mp / C::BM) * (g.Np / C::BN) * splits;
  TimedLaunch tl(kKcGemmStore, s);
  if (g.pk && g.qk) store_launch<C, T, true, true>(a, tiles, C0, C1, msplit, ldc, slab, bias, bn, s);
  else if (g.pk && !g.qk) store_launch<C, T, true, false>(a, tiles, C0, C1, msplit, ldc, slab, bias, bn, s);
  else if (!g.pk && !g.qk) store_launch<C, T, false, false>(a, tiles, C0, C1, msplit, ldc, slab, bias, bn, s);
  else throw Gm2Error("gemm: layout (P MN-major, Q K-major) not instantiated");
  GM2_CHECK_LAUNCH();
  return splits;
}

template <typename T>
int launch_gemm_store(const GemmArgs<T>& g, int splits, float* C0, float* C1, int msplit, int64_t ldc, int64_t slab,
                      const float* bias, hipStream_t s) {
  if (splits < 0) splits = plan_gemm(g).splits;
  const StoreEpi none{};
  if constexpr (sizeof(T) == 2) {  // (256x256 tiles: bf16 only, see plan_gemm)
    if (use_big(g)) {
      check_gemm(g, 256);
      return store_impl<Big, T>(g, splits, C0, C1, msplit, ldc, slab, bias, none, s);
    }
  }
  check_gemm(g, 128);
  return small_cfg<T>([&](auto cfg) { return store_impl<decltype(cfg), T>(g, splits, C0, C1, msplit, ldc, slab, bias, none, s); });
}

template <typename T>
int gemm_tiles(const GemmArgs<T>& g) {
  return use_big(g) ? (g.Mp / Big::BM) * (g.Np / Big::BN) : (g.Mp / SmallDeep::BM) * (g.Np / SmallDeep::BN);
}

template <typename T>
bool launch_gemm_sq(const GemmArgs<T>& g, float* C, int64_t ldc, double* sq, hipStream_t s, bool force_big) {
  // force_big: a one-pass 256x256-tile launch even where the plan would pick 128 tiles (a row
  // slice of a big-tile GEMM, same per-element results as the whole)
  const bool big = force_big ? (sizeof(T) == 2 && g.Mp % 256 == 0 && g.Np % 256 == 0) : use_big(g);
  if (!force_big && plan_gemm(g).splits != 1) return false;
  if (force_big && !big) return false;
  StoreEpi ep;
  ep.sq = sq;
  ep.ntiles = (grid_cap_bits() & 2) && !force_big;  // dWe0 bit
  if constexpr (sizeof(T) == 2) {
    if (big) {
      check_gemm(g, 256);
      store_impl<Big, T>(g, 1, C, nullptr, 0, ldc, 0, nullptr, ep, s);
      return true;
    }
  }
  check_gemm(g, 128);
  small_cfg<T>([&](auto cfg) { return store_impl<decltype(cfg), T>(g, 1, C, nullptr, 0, ldc, 0, nullptr, ep, s); });
  return true;
}

template <typename T>
bool launch_gemm_trans(const GemmArgs<T>& g, float* C, int64_t ldc, hipStream_t s, double* sq) {
  if (plan_gemm(g).splits != 1) return false;
  StoreEpi ep;
  ep.trans = 1;
  ep.sq = sq;

  ep.ntiles = grid_cap_bits() & 1;  // dW9 bit (the launcher sets the count)
  if constexpr (sizeof(T) == 2) {
    if (use_big(g)) {
      check_gemm(g, 256);
      store_impl<Big, T>(g, 1, C, nullptr, 0, ldc, 0, nullptr, ep, s);
      return true;
    }
  }
  check_gemm(g, 128);
  small_cfg<T>([&](auto cfg) { return store_impl<decltype(cfg), T>(g, 1, C, nullptr, 0, ldc, 0, nullptr, ep, s); });
  return true;
}

// BatchNorm statistics in the store epilogue (GM2_OPT_BN_EPILOGUE, default on): taken when the
// plan is one pass of 128-row tiles (the statistics chunk), else the caller runs the separate pass


template <typename T>
bool launch_gemm_bn(const GemmArgs<T>& g, float* C, int64_t ldc, const float* bias, const StoreEpi& bn, hipStream_t s) {
  static_assert(Small::BM == kBnRowChunk, "statistics chunk = row tile");
  if (!opts().bn_epilogue) return false;
  const GemmPlan p = plan_gemm(g);
  if (p.tile != 128 || p.splits != 1 || (bn.mode && (g.N % 4 || bn.ldy % 4))) return false;
  check_gemm(g, 128);
  small_cfg<T>([&](auto cfg) { return store_impl<decltype(cfg), T>(g, 1, C, nullptr, 0, ldc, 0, bias, bn, s); });
  return true;
}

template <typename T>
static bool recon_big(const GemmArgs<T>& g);

template <typename T>
int gemm_recon_grid_blocks(const GemmArgs<T>& g) {
  const int t = recon_big(g) ? 256 : 128;
  return (g.Np / t) * (g.Mp / t);
}

template <typename T>
int gemm_recon_row_tiles(const GemmArgs<T>& g) {  // strain tiles (rows of colpart)
  return g.Np / (recon_big(g) ? 256 : 128);
}

template <class C, typename T, bool PP>
static void recon_impl_k(const GemmArgs<T>& g, const float* bias, const uint32_t* X, int64_t ldx, int with_grad,
                         const float* scal, T* dL, int64_t ldd, float* loss_part, float* colpart, int64_t ldcol,
                         hipStream_t s, const int32_t* xrows) {
  check_gemm(g, C::BM);
  if (ldx * 32 < g.Mp || (ldx & 3)) throw Gm2Error("recon: target bit rows too short");
  constexpr int lds = recon_lds_bytes<C, T>();
  static_assert(lds <= 160 * 1024, "LDS budget");
  const int tiles = (g.Mp / C::BM) * (g.Np / C::BN);
  int grid = tiles, ntiles = 0;
  if (grid_cap_bits() & 4) {  // same rounds on fewer workgroups
    const int cus = device_cus(), rounds = (tiles + cus - 1) / cus;
    grid = (tiles + rounds - 1) / rounds;
    ntiles = grid < tiles ? tiles : 0;
  }
  auto go = [&](auto kern) {
    ensure_lds_attr((const void*)kern, lds);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(C::NT), lds, s, g, bias, X, ldx, ntiles, scal, dL, ldd, loss_part,
                       colpart, ldcol, xrows);
  };
  if (with_grad) go(k_gemm_recon_loss<C, T, PP, true>);
  else go(k_gemm_recon_loss<C, T, PP, false>);
}

template <class C, typename T>
static void recon_impl(const GemmArgs<T>& g, const float* bias, const uint32_t* X, int64_t ldx, int with_grad,
                       const float* scal, T* dL, int64_t ldd, float* loss_part, float* colpart, int64_t ldcol,
                       hipStream_t s, const int32_t* xrows) {
  if constexpr (std::is_same_v<C, Big> && sizeof(T) == 2) {
    if (pp_enabled())
      return recon_impl_k<C, T, true>(g, bias, X, ldx, with_grad, scal, dL, ldd, loss_part, colpart, ldcol, s, xrows);
  }
  recon_impl_k<C, T, false>(g, bias, X, ldx, with_grad, scal, dL, ldd, loss_part, colpart, ldcol, s, xrows);
}

// the fp32 parity path stays on the 128-tile (a 256-row fp32 dL image would not fit the LDS).
// GM2_OPT_RECON_TILE: 0 = plan (256 when it fills the chip), 128 / 256 = force (A/B measurements)


template <typename T>
static bool recon_big(const GemmArgs<T>& g) {
  const int force = opts().recon_tile;
  const bool ok = sizeof(T) == 2 && g.Mp % 256 == 0 && g.Np % 256 == 0;
  if (force == 128) return false;
  if (force == 256) return ok;
  return ok && (g.Mp / 256) * (g.Np / 256) >= 128;
}

template <typename T>
void launch_gemm_recon_loss(const GemmArgs<T>& g, const float* bias, const uint32_t* X, int64_t ldx, int with_grad,
                            const float* scal, T* dL, int64_t ldd, float* loss_part, float* colpart, int64_t ldcol,
                            hipStream_t s, const int32_t* xrows) {
  TimedLaunch tl(kKcReconLoss, s);
  bool done = false;
  if constexpr (sizeof(T) == 2) {
    if (recon_big(g)) {
      recon_impl<Big, T>(g, bias, X, ldx, with_grad, scal, dL, ldd, loss_part, colpart, ldcol, s, xrows);
      done = true;
    }
  }
  if (!done) recon_impl<Small, T>(g, bias, X, ldx, with_grad, scal, dL, ldd, loss_part, colpart, ldcol, s, xrows);
  GM2_CHECK_LAUNCH();
}

template <typename T>
bool gemm_idx_ok(const GemmArgs<T>& g) {
  if (sizeof(T) != 2 || !pp_enabled()) return false;
  const GemmPlan p = plan_gemm<T>(g);
  if (p.tile != 256) return false;
  if (!g.qrow) return true;  // (P rows: one 256-row table per tile)
  const int nkt = g.K / E<T>::KT, splits = std::max(1, std::min(p.splits, nkt));
  const int kps = (int)(round_up(nkt, splits) / splits) * E<T>::KT;
  return kps <= kMaxIdxRows;  // (Q k-rows: a split's k-rows in the table)
}

void launch_gemm_mask_tiered(const GemmArgs<bf16_t>& g1, const GemmArgs<bf16_t>& g3, const float* bias, uint8_t* mask,
                             int64_t ldm, uint8_t* bits, int64_t ldb, hipStream_t s, MaskGate gate1, MaskBand band1,
                             MaskGate gate3, MaskBand band3) {
  check_gemm(g1, 256);
  check_gemm(g3, 256);
  if (g1.Mp != g3.Mp || g1.Np != g3.Np || g1.Mp % 256 || g1.Np % 256 || g1.K % 64 || g3.K % 64)
    throw Gm2Error("tiered mask: the two GEMMs' tile grids differ");
  if (bits && ((ldb & 15) || (((uintptr_t)bits) & 15) || ldb * 8 < g3.N))
    throw Gm2Error("mask bits: row pitch %lld must be a multiple of 16 bytes covering the padded genes", (long long)ldb);
  if (!band1.rn || !band3.rn || !band1.tslots || !band3.tslots || !band1.drop_overflow || !gate3.run)
    throw Gm2Error("tiered mask: both bands with tile slots (the single tier's dropping its overflow) and the gate");
  if (!band3.oflag || !band3.olist || !band3.ocount || band3.obn < g3.Np / 256 ||
      band3.oblocks < (unsigned)((g3.Mp / 256) * band3.obn))
    throw Gm2Error("tiered mask: the overflow block flags, list and counter required");
  const MaskOut o1{mask, ldm, bits, ldb, nullptr, 0, nullptr, nullptr, 0, 0.5f, gate1, band1};
  const MaskOut o3{mask, ldm, bits, ldb, nullptr, 0, nullptr, nullptr, 0, 0.5f, gate3, band3};
  constexpr int lds = Big::LDS + band_lds_bytes<Big>();
  const dim3 grid((g3.Mp / 256) * (g3.Np / 256));
  TimedLaunch tl(kKcMask, s);
  auto go = [&](auto kern) {
    ensure_lds_attr((const void*)kern, lds);
    hipLaunchKernelGGL(kern, grid, dim3(Big::NT), lds, s, g1, g3, bias, o1, o3);
  };
  // (packed bits and u8 masks both leave the bit-image epilogue: its ballots replace the byte image's
  // per-element LDS stores; the u8 form through k_gemm_mask_tiered<..., false> measured 11.7 vs 5.3 ms
  // per 65,536-genome chunk, profiles/r06_decode_u8_ab.txt)
  go(k_gemm_mask_tiered<Big, bf16_t, true>);
  GM2_CHECK_LAUNCH();
}

template <typename T>
void launch_gemm_mask(const GemmArgs<T>& g, const float* bias, uint8_t* mask, int64_t ldm, float* probs, int64_t ldpr,
                      hipStream_t s, uint8_t* bits, int64_t ldb, int* counts, const uint32_t* xbits, int64_t ldxb,
                      float thr, bool big, MaskGate gate, MaskBand band) {
  check_gemm(g, big ? 256 : 128);
  // (the 256-column tiles may reach past the row pitch: their bits stores stop at ldb, past G)
  if (bits && ((ldb & 15) || (((uintptr_t)bits) & 15) || ldb * 8 < (big ? g.N : g.Np)))
    throw Gm2Error("mask bits: row pitch %lld must be a multiple of 16 bytes covering the padded genes", (long long)ldb);
  if (counts && (!xbits || ldxb * 32 < g.Np)) throw Gm2Error("mask counts: target bits required");
  MaskOut o{mask, ldm, bits, ldb, probs, ldpr, counts, xbits, ldxb, thr, gate, band};
  if (band.rn && (!band.cn || !band.counts || !band.list || !band.cap || thr != 0.5f))
    throw Gm2Error("mask band: norms, counter and list required (threshold 0.5 only)");
  if (band.rn && (!band.oflag || !band.olist || !band.ocount || band.obn < (g.Np + 255) / 256 ||
                  band.oblocks < (unsigned)(((g.Mp + 255) / 256) * band.obn)))
    throw Gm2Error("mask band: the overflow block flags, list and counter required");
  if (band.tslots && (!band.tlist || !band.tcount || !band.tfound || !big))
    throw Gm2Error("mask band: tile slots need their list, counters and the 256 x 256 kernel");
  const int band_lds = band.rn ? (big ? band_lds_bytes<Big>() : band_lds_bytes<Small>()) : 0;  // (norms + slot counter)
  TimedLaunch tl(kKcMask, s);
  if constexpr (sizeof(T) == 2) {
    if (big) {
      if (g.Mp % 256 || g.Np % 256 || g.K % 64) throw Gm2Error("mask (256x256): padded extents");
      static_assert(Big::LDS >= 256 * (256 + 16), "u8 image inside the staging ring");
      constexpr int lds_max = Big::LDS + band_lds_bytes<Big>();
      const int lds = Big::LDS + band_lds;
      const dim3 grid((g.Mp / 256) * (g.Np / 256));
      auto go = [&](auto kern) {
        ensure_lds_attr((const void*)kern, lds_max);
        hipLaunchKernelGGL(kern, grid, dim3(Big::NT), lds, s, g, bias, o);
      };
      const bool ballot = bits && !mask && !probs && !counts && thr == 0.5f;  // packed bits only: ballot epilogue
      if (ballot) go(k_gemm_mask<Big, T, true, true>);
      else go(k_gemm_mask<Big, T, true>);
      GM2_CHECK_LAUNCH();
      return;
    }
  }
  if (big) throw Gm2Error("mask (256x256): bf16 only");
  static_assert(Small::LDS >= 128 * (128 + 16), "u8 image inside the staging ring");
  const int ntile = (g.Mp / 128) * (g.Np / 128);
  if (gate.run) {  // (the tile loop, from a grid of at most 1024 workgroups)
    // (LDS: the band region always, then the verdict words)
    constexpr int lds = Small::LDS + band_lds_bytes<Small>() + (Small::NT / 64) * 8;
    ensure_lds_attr((const void*)k_gemm_mask<Small, T, false, false, true>, lds);
    hipLaunchKernelGGL((k_gemm_mask<Small, T, false, false, true>), dim3(std::min(ntile, 1024)), dim3(Small::NT), lds,
                       s, g, bias, o);
  } else {
    if (band_lds) ensure_lds_attr((const void*)k_gemm_mask<Small, T>, Small::LDS + band_lds_bytes<Small>());
    hipLaunchKernelGGL((k_gemm_mask<Small, T>), dim3(ntile), dim3(Small::NT), Small::LDS + band_lds, s, g, bias, o);
  }
  GM2_CHECK_LAUNCH();
}

#define GM2_INST(T)                                                                                              \
  template bool launch_gemm_trans<T>(const GemmArgs<T>&, float*, int64_t, hipStream_t, double*);                    \
  template bool launch_gemm_sq<T>(const GemmArgs<T>&, float*, int64_t, double*, hipStream_t, bool);                \
  template int gemm_tiles<T>(const GemmArgs<T>&);                        \
  template bool launch_gemm_bn<T>(const GemmArgs<T>&, float*, int64_t, const float*, const StoreEpi&, hipStream_t);   \
  template int launch_gemm_store<T>(const GemmArgs<T>&, int, float*, float*, int, int64_t, int64_t, const float*, \
                                    hipStream_t);                                                                \
  template int gemm_recon_grid_blocks<T>(const GemmArgs<T>&);                                                   \
  template int gemm_recon_row_tiles<T>(const GemmArgs<T>&);                                                     \
  template GemmPlan plan_gemm<T>(const GemmArgs<T>&);                                                          \
  template void launch_gemm_recon_loss<T>(const GemmArgs<T>&, const float*, const uint32_t*, int64_t, int,        \
                                          const float*, T*, int64_t, float*, float*, int64_t, hipStream_t,      \
                                          const int32_t*);                                                      \
  template bool gemm_idx_ok<T>(const GemmArgs<T>&);
GM2_INST(float)
GM2_INST(bf16_t)
#undef GM2_INST
template void launch_gemm_mask<float>(const GemmArgs<float>&, const float*, uint8_t*, int64_t, float*, int64_t,
                                      hipStream_t, uint8_t*, int64_t, int*, const uint32_t*, int64_t, float, bool,
                                      MaskGate, MaskBand);
template void launch_gemm_mask<bf16_t>(const GemmArgs<bf16_t>&, const float*, uint8_t*, int64_t, float*, int64_t,
                                       hipStream_t, uint8_t*, int64_t, int*, const uint32_t*, int64_t, float, bool,
                                       MaskGate, MaskBand);

#ifdef GM2_DEBUG
GM2_DBG_TAKE_FN(dbg_take_gemm)
#endif

}  // namespace gm2
