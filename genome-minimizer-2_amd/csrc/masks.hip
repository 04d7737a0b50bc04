// Consumers of the sampled masks, on the packed masks in HBM:
//   * count_essential_genes (utils/extras.py:49-87): per sample, the number of essential genes
//     present, a gene counting when ANY of its column positions is set;
//   * masks_to_gene_lists (explore_data/binary_converter.py:19-76): per sample, the ascending
//     column indices of the set genes (duplicate gene names dropped through a keep mask), as a
//     CSR (row offsets = exclusive scan of row popcounts, then a wave-parallel compaction).
// Mask rows are numpy packbits(bitorder='little') bytes: bit (g & 7) of byte g / 8 = gene g,
// row pitch ld_bits (multiple of 16 bytes), bits beyond G zero. HBM-bound integer work: every
// kernel streams each mask row once with 16-byte (or 4-byte word) loads.
#include "../../include/gm2.h"
#include "gm2_common.hpp"
#include "gm2_kernels.hpp"

namespace gm2 {

namespace {

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// one wave per sample row; lane l evaluates groups l, l+64, ...: a group counts when any of its
// positions is set (the reference's `break` after the first present position)
__global__ __launch_bounds__(256) void k_count_groups(const uint8_t* __restrict__ bits, int64_t n, int64_t ldb,
                                                    const int32_t* __restrict__ goff, int ngroups,
                                                    const int32_t* __restrict__ pos, int32_t* __restrict__ counts) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const uint8_t* r = bits + row * ldb;
  int cnt = 0;
  for (int gi = lane; gi < ngroups; gi += 64) {
    int any = 0;
    GM2_DBG(goff[gi] >= 0 && goff[gi] <= goff[gi + 1], kDbgMaskPos);
    for (int k = goff[gi]; k < goff[gi + 1] && !any; ++k) {
      const int p = pos[k];
      GM2_DBG(p >= 0 && (int64_t)(p >> 3) < ldb, kDbgMaskPos);
      any = (r[p >> 3] >> (p & 7)) & 1;
    }
    cnt += any;
  }
  cnt = wave_sum_i(cnt);
  if (lane == 0) counts[row] = cnt;
}

// The same count from whole-row reads: each workgroup first turns the groups into an LDS bit mask of
// the single-position groups (one atomicOr per group; a position already in the mask -- a second
// group on the same gene -- and every multi-position group go to an LDS list instead), then its
// waves stream their rows with 16-byte loads: count = popcount(row AND mask) + the listed groups
// evaluated as above. The same integer as k_count_groups; a row's ~300 scattered byte reads touched
// nearly every line of the row anyway, now one coalesced pass reads it.
constexpr int kCountRowsPerWg = 16;
__global__ __launch_bounds__(256) void k_count_groups_rows(const uint8_t* __restrict__ bits, int64_t n, int64_t ldb,
                                                         const int32_t* __restrict__ goff, int ngroups,
                                                         const int32_t* __restrict__ pos, int32_t* __restrict__ counts,
                                                         int stage) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lmask[];  // [ldb / 4] words, then the list
  const int nw = (int)(ldb / 4);
  int* glist = (int*)(lmask + nw);
  int* gcount = glist + ngroups;
  // (stage: each wave keeps the row it streams in an LDS row buffer [4][ldb], and the listed groups'
  // byte reads go there instead of back to global memory -- they were ~4x the rows' own bytes)
  uint8_t* wrow = (uint8_t*)lmask + ((ldb + (int64_t)(ngroups + 1) * 4 + 15) & ~(int64_t)15) +
                  (int64_t)(threadIdx.x >> 6) * ldb;
  for (int i = threadIdx.x; i < nw; i += 256) lmask[i] = 0u;
  if (threadIdx.x == 0) *gcount = 0;
  __syncthreads();
  for (int g = threadIdx.x; g < ngroups; g += 256) {
    const int k0 = goff[g], k1 = goff[g + 1];
    GM2_DBG(k0 >= 0 && k0 <= k1, kDbgMaskPos);
    if (k1 == k0) continue;  // (an empty group never counts)
    if (k1 - k0 == 1) {
      const int p = pos[k0];
      GM2_DBG(p >= 0 && (int64_t)(p >> 3) < ldb, kDbgMaskPos);
      const uint32_t bit = 1u << (p & 31);
      if (!(atomicOr(&lmask[p >> 5], bit) & bit)) continue;
    }
    glist[atomicAdd(gcount, 1)] = g;
  }
  __syncthreads();
  const int ng = *gcount, lane = threadIdx.x & 63;
  const int64_t r1 = min(n, (int64_t)(blockIdx.x + 1) * kCountRowsPerWg);
  for (int64_t row = (int64_t)blockIdx.x * kCountRowsPerWg + (threadIdx.x >> 6); row < r1; row += 4) {
    const uint8_t* rb = bits + row * ldb;
    const uint4* r = (const uint4*)rb;
    const uint4* m = (const uint4*)lmask;
    int c = 0;
    // (four 16-byte loads per lane in flight before their first use)
    for (int i0 = lane; i0 < nw / 4; i0 += 4 * 64) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = i0 + u * 64 < nw / 4 ? r[i0 + u * 64] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (i0 + u * 64 >= nw / 4) break;
        if (stage) ((uint4*)wrow)[i0 + u * 64] = v[u];
        const uint4 k = m[i0 + u * 64];
        c += __builtin_popcount(v[u].x & k.x) + __builtin_popcount(v[u].y & k.y) +
             __builtin_popcount(v[u].z & k.z) + __builtin_popcount(v[u].w & k.w);
      }
    }
    const uint8_t* lb = stage ? wrow : rb;
    if (stage) {  // (this wave's row writes, visible to its own lanes' reads below)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    }
    for (int j = lane; j < ng; j += 64) {
      const int g = glist[j];
      int any = 0;
      for (int k = goff[g]; k < goff[g + 1] && !any; ++k) {
        const int p = pos[k];
        GM2_DBG(p >= 0 && (int64_t)(p >> 3) < ldb, kDbgMaskPos);
        any = (lb[p >> 3] >> (p & 7)) & 1;
      }
      c += any;
    }
    if (stage) __builtin_amdgcn_wave_barrier();  // (the next row overwrites the buffer after these reads)
    c = wave_sum_i(c);
    if (lane == 0) counts[row] = c;
  }
}

// popcount of each row (AND keep mask) -> out[row]; one wave per row, 16-byte loads
__global__ __launch_bounds__(256) void k_row_popcount(const uint8_t* __restrict__ bits, int64_t n, int64_t ldb,
                                                    const uint8_t* __restrict__ keep, int64_t* __restrict__ out) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const uint4* r = (const uint4*)(bits + row * ldb);
  const uint4* kp = (const uint4*)keep;
  int c = 0;
  for (int64_t i = lane; i < ldb / 16; i += 64) {
    uint4 v = r[i];
    if (kp) {
      const uint4 k = kp[i];
      v.x &= k.x; v.y &= k.y; v.z &= k.z; v.w &= k.w;
    }
    c += __builtin_popcount(v.x) + __builtin_popcount(v.y) + __builtin_popcount(v.z) + __builtin_popcount(v.w);
  }
  c = wave_sum_i(c);
  if (lane == 0) out[row] = c;
}

// in-place inclusive scan of a[0..n) (int64), one workgroup of 1024 threads: per-thread chunk sums,
// an LDS scan of the 1024 sums, then each chunk rewritten with its offset
__global__ __launch_bounds__(1024) void k_scan_inclusive(int64_t* __restrict__ a, int64_t n) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x;
  const int64_t chunk = (n + 1023) / 1024;
  const int64_t lo = t * chunk, hi = min(n, lo + chunk);
  int64_t s = 0;
  for (int64_t i = lo; i < hi; ++i) s += a[i];
  part[t] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int64_t v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int64_t run = t ? part[t - 1] : 0;
  for (int64_t i = lo; i < hi; ++i) {
    run += a[i];
    a[i] = run;
  }
}

// set-bit column indices of each row in ascending order at out[off[row] ...]: one wave per row,
// 64 words per pass (lane l holds word base + l), exclusive wave scan of the word popcounts
__global__ __launch_bounds__(256) void k_compact(const uint8_t* __restrict__ bits, int64_t n, int64_t ldb,
                                               const uint8_t* __restrict__ keep, const int64_t* __restrict__ off,
                                               int32_t* __restrict__ idx) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const uint32_t* r = (const uint32_t*)(bits + row * ldb);
  const uint32_t* kp = (const uint32_t*)keep;
  int64_t out = off[row];
  const int64_t nw = ldb / 4;
  for (int64_t base = 0; base < nw; base += 64) {
    const int64_t wi = base + lane;
    uint32_t w = wi < nw ? r[wi] : 0u;
    if (kp && wi < nw) w &= kp[wi];
    const int c = __builtin_popcount(w);
    int pre = c;  // inclusive scan over the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(pre, o, 64);
      if (lane >= o) pre += v;
    }
    const int tot = __shfl(pre, 63, 64);
    int64_t dst = out + pre - c;
    while (w) {
      const int b = __builtin_ctz(w);
      GM2_DBG(dst >= off[row] && dst < off[row + 1], kDbgCompact);
      idx[dst++] = (int32_t)(wi * 32 + b);
      w &= w - 1;
    }
    out += tot;
  }
}

}  // namespace

void launch_count_groups(const uint8_t* bits, int64_t n, int64_t ldb, const int32_t* goff, int64_t ngroups,
                         const int32_t* pos, int32_t* counts, hipStream_t s) {
  if (n <= 0) return;
  // (whole-row form when the rows are 16-B pieces and the mask + list fit in 64 KB of LDS; each wave's
  // row buffer too when that still fits)
  const int64_t lds = ldb + (ngroups + 1) * 4;
  const int64_t lds_stage = ((lds + 15) & ~(int64_t)15) + 4 * ldb;
  if ((ldb & 15) == 0 && (((uintptr_t)bits) & 15) == 0 && lds <= 64 * 1024) {
    const int stage = lds_stage <= 64 * 1024 ? 1 : 0;
    hipLaunchKernelGGL(k_count_groups_rows, dim3((unsigned)((n + kCountRowsPerWg - 1) / kCountRowsPerWg)), dim3(256),
                       (unsigned)(stage ? lds_stage : lds), s, bits, n, ldb, goff, (int)ngroups, pos, counts, stage);
  } else {
    hipLaunchKernelGGL(k_count_groups, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, bits, n, ldb, goff,
                       (int)ngroups, pos, counts);
  }
  GM2_CHECK_LAUNCH();
}

void launch_row_offsets(const uint8_t* bits, int64_t n, int64_t ldb, const uint8_t* keep, int64_t* offsets,
                        hipStream_t s) {
  if (hipMemsetAsync(offsets, 0, sizeof(int64_t), s) != hipSuccess) throw Gm2Error("hipMemsetAsync");
  if (n <= 0) return;
  hipLaunchKernelGGL(k_row_popcount, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, bits, n, ldb, keep, offsets + 1);
  GM2_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_scan_inclusive, dim3(1), dim3(1024), 0, s, offsets + 1, n);
  GM2_CHECK_LAUNCH();
}

void launch_compact(const uint8_t* bits, int64_t n, int64_t ldb, const uint8_t* keep, const int64_t* offsets,
                    int32_t* idx, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_compact, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, bits, n, ldb, keep, offsets, idx);
  GM2_CHECK_LAUNCH();
}

#ifdef GM2_DEBUG
GM2_DBG_TAKE_FN(dbg_take_masks)
#endif

}  // namespace gm2
