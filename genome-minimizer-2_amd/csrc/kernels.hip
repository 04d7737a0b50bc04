// Non-GEMM kernels of the VAE hot path: strain-row gather, BatchNorm (train/eval, fwd/bwd),
// reparameterization + KL, deterministic reductions, clip-norm statistics, Adam, GEMM shadows.
// All are HBM/latency-bound streaming kernels over [B,H]-sized (or P-sized) data; they keep
// every padded element of their outputs at zero (the GEMM operand contract, gemm.hip).
#include "bn_common.hpp"
#include "gm2_common.hpp"
#include "gm2_kernels.hpp"

namespace gm2 {

namespace {

static_assert(kBnChunk == kBnRowChunk, "BatchNorm chunk size");

// ---------------------------------------------------------------------------------------------
// gather: X[r][c] = data[rows[r]][c] (u8, nonzero -> 1, as T) and the row-major target bits of the
// loss epilogue (bit c%32 of word c/32 of row r). A wave streams 8 strain rows: 8 bytes per lane =
// 512 contiguous bytes per load instruction, all 8 rows' loads in flight, then one lane-contiguous
// store per row (1 KiB bf16 / 2 KiB f32 per instruction); block = 4 waves x 8 rows x 512 columns.
// Each lane's 8 columns are one byte of a target word; lane 4j writes word j of its 128-column
// group. Rows and X stream (non-temporal: read once here, X re-read by the input-layer GEMMs).
// ---------------------------------------------------------------------------------------------
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;

// bytes -> 0x00 / 0x01 (nonzero -> 1): OR-fold each byte into its bit 0 (no cross-byte leaks
// reach bit 0: every shift source of bit 0 of byte k is a bit of byte k)
__device__ __forceinline__ uint32_t bytes_to_01(uint32_t x) {
  x |= x >> 4;
  x |= x >> 2;
  x |= x >> 1;
  return x & 0x01010101u;
}

template <typename T>
__global__ __launch_bounds__(256) void k_gather(const uint8_t* __restrict__ data, int64_t ld_data,
                                              const int32_t* __restrict__ rows, int B, int G, int Gp,
                                              T* __restrict__ X, int64_t ldx, uint32_t* __restrict__ xbits,
                                              int64_t ldxb) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = blockIdx.x * 512 + lane * 8;
  const int rbase = blockIdx.y * 32 + wid * 8;
  const bool in = c < Gp;  // Gp % 128 == 0: whole 4-lane word groups are in or out
  // reads stop at the lane group holding gene G-1 (ld_data >= roundup(G, 128) is all the caller
  // promises, while Gp may be padded further, to 256, for the bf16 GEMM tiles)
  const bool rd = c < G;
  u32x2 v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int r = rbase + k;
    v[k] = u32x2{0u, 0u};
    if (rd && r < B) {
      const int64_t src = rows ? (int64_t)rows[r] : (int64_t)r;
      GM2_DBG(src >= 0, kDbgGatherRows);
      v[k] = __builtin_nontemporal_load((const u32x2*)(data + src * ld_data + c));
    }
  }
  // columns >= G read as zero (the resident matrix's pad is zero already; this keeps X's pad zero
  // whatever ld_data holds there)
  const uint32_t keep0 = c + 4 <= G ? 0xFFFFFFFFu : (c >= G ? 0u : (0xFFFFFFFFu >> (8 * (c + 4 - G))));
  const uint32_t keep1 = c + 8 <= G ? 0xFFFFFFFFu : (c + 4 >= G ? 0u : (0xFFFFFFFFu >> (8 * (c + 8 - G))));
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int r = rbase + k;
    const uint32_t t0 = bytes_to_01(v[k][0]) & keep0, t1 = bytes_to_01(v[k][1]) & keep1;
    if (in) {
      T* dst = X + (int64_t)r * ldx + c;
      if constexpr (sizeof(T) == 2) {
        // (b1 << 16 | b0) * 0x3F80 = the two bf16 values (1.0 = 0x3F80), no carries for b in {0,1}
        const uint32_t w0 = __builtin_amdgcn_perm(0u, t0, 0x0c010c00u) * 0x3F80u;
        const uint32_t w1 = __builtin_amdgcn_perm(0u, t0, 0x0c030c02u) * 0x3F80u;
        const uint32_t w2 = __builtin_amdgcn_perm(0u, t1, 0x0c010c00u) * 0x3F80u;
        const uint32_t w3 = __builtin_amdgcn_perm(0u, t1, 0x0c030c02u) * 0x3F80u;
        __builtin_nontemporal_store(u32x4{w0, w1, w2, w3}, (u32x4*)dst);
      } else {
        *(float4*)dst = make_float4((float)(t0 & 1), (float)((t0 >> 8) & 1), (float)((t0 >> 16) & 1), (float)(t0 >> 24));
        *(float4*)(dst + 4) = make_float4((float)(t1 & 1), (float)((t1 >> 8) & 1), (float)((t1 >> 16) & 1), (float)(t1 >> 24));
      }
    }
    if (xbits) {
      // byte b_i (0/1) at bit 8i -> bit i: (t * 0x01020408) >> 24 collects them without carries
      const uint32_t b8 = ((t0 * 0x01020408u) >> 24 & 0xFu) | (((t1 * 0x01020408u) >> 24 & 0xFu) << 4);
      const uint32_t w = b8 | (__shfl_down(b8, 1, 64) << 8) | (__shfl_down(b8, 2, 64) << 16) |
                         (__shfl_down(b8, 3, 64) << 24);
      if (in && (lane & 3) == 0) xbits[(int64_t)r * ldxb + (c >> 5)] = w;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// BN forward partial statistics of Y = sum of S split-K slabs + bias (the GEMMs whose plan is not
// one 128-row-tile pass; the others take them in their epilogue). Block: 64 columns x one 128-row
// chunk; thread = 4 columns (float4) x 8 rows (16 row groups), all 8 rows' loads of a slab in
// flight together; two-pass (mean, M2) per chunk.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float4 f4add(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }

__global__ __launch_bounds__(256) void k_bn_fwd_partial(const float* __restrict__ slabs, int S, int64_t slab,
                                                      int64_t ld, const float* __restrict__ bias, int B, int H,
                                                      float* __restrict__ Y, float2* __restrict__ part) {
  __shared__ float4 red[16][16];
  const int cg = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int col = blockIdx.x * 64 + cg * 4;
  const int r0 = blockIdx.y * kBnRowChunk;
  const int nrows = min(kBnRowChunk, B - r0);
  const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 b = bias ? *(const float4*)(bias + col) : zero;
  // rows past nrows re-read the chunk's last row (never used): branch-free loads, and up to four
  // slabs' loads in flight together
  float4 v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = *(const float4*)(slabs + (int64_t)(r0 + min(rg + 16 * i, nrows - 1)) * ld + col);
  for (int sl = 1; sl < S; sl += 3) {
    float4 w[3][8];
#pragma unroll
    for (int u = 0; u < 3; ++u)
      if (sl + u < S)
#pragma unroll
        for (int i = 0; i < 8; ++i)
          w[u][i] = *(const float4*)(slabs + (int64_t)(sl + u) * slab + (int64_t)(r0 + min(rg + 16 * i, nrows - 1)) * ld + col);
#pragma unroll
    for (int u = 0; u < 3; ++u)
      if (sl + u < S)
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = f4add(v[i], w[u][i]);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = f4add(v[i], b);
  // the chunk mean from sums of (v - shift), shift = the chunk's first row (a sample of the column):
  // |v - shift| ~ the column's spread, not its mean, so the fp32 sum keeps the mean accurate to a
  // few ulps of the spread -- what the backward's near-cancelling sum((y - mean) do) needs (the
  // GEMM-epilogue statistics use the same shift)
  if (rg == 0) red[0][cg] = v[0];
  __syncthreads();
  const float4 sh = red[0][cg];
  __syncthreads();
  float4 sum = zero;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int rl = rg + 16 * i;
    if (rl < nrows) {
      *(float4*)(Y + (int64_t)(r0 + rl) * ld + col) = v[i];
      sum = f4add(sum, make_float4(v[i].x - sh.x, v[i].y - sh.y, v[i].z - sh.z, v[i].w - sh.w));
    }
  }
  red[rg][cg] = sum;
  __syncthreads();
  float4 tot = zero;
#pragma unroll
  for (int k = 0; k < 16; ++k) tot = f4add(tot, red[k][cg]);
  const float inv = 1.f / (float)nrows;
  const float4 mean = make_float4(fmaf(tot.x, inv, sh.x), fmaf(tot.y, inv, sh.y), fmaf(tot.z, inv, sh.z),
                                  fmaf(tot.w, inv, sh.w));
  __syncthreads();
  float4 m2 = zero;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (rg + 16 * i < nrows) {
      const float dx = v[i].x - mean.x, dy = v[i].y - mean.y, dz = v[i].z - mean.z, dw = v[i].w - mean.w;
      m2 = make_float4(fmaf(dx, dx, m2.x), fmaf(dy, dy, m2.y), fmaf(dz, dz, m2.z), fmaf(dw, dw, m2.w));
    }
  }
  red[rg][cg] = m2;
  __syncthreads();
  if (rg == 0) {
    float4 q = zero;
#pragma unroll
    for (int k = 0; k < 16; ++k) q = f4add(q, red[k][cg]);
    float4* o = (float4*)(part + (int64_t)blockIdx.y * H + col);
    o[0] = make_float4(mean.x, q.x, mean.y, q.y);
    o[1] = make_float4(mean.z, q.z, mean.w, q.w);
  }
}

// Chan's parallel merge of per-chunk (mean, M2) -> batch mean and biased variance, in two passes
// (mean = sum n_c mean_c / B ; M2 = sum M2_c + n_c (mean_c - mean)^2), fp64. Up to 32 chunks
// (B <= 4096) the partials are loaded once, all in flight, and both passes run from registers.
__device__ __forceinline__ void bn_merge(const float2* __restrict__ part, int B, int H, int col, double& mean, double& var) {
  bn_merge_ld([&](int ch) { return part[(int64_t)ch * H + col]; }, B, mean, var);
}

// ---------------------------------------------------------------------------------------------
// BN backward partials: do = dA * [y*alpha+beta' > 0] with dA = sum of S slabs (written to dsum when
// S > 1); sums of do and (y-mean)*do per 128-row chunk. Same block shape as k_bn_fwd_partial.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_bn_bwd_partial(const float* __restrict__ dslabs, int S, int64_t slab,
                                                      const float* __restrict__ Y, int64_t ld,
                                                      const float* __restrict__ save, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, int B, int H,
                                                      float2* __restrict__ part, float* __restrict__ dsum) {
  __shared__ float4 red[2][16][16];
  const int cg = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int col = blockIdx.x * 64 + cg * 4;
  const int r0 = blockIdx.y * kBnRowChunk;
  const int nrows = min(kBnRowChunk, B - r0);
  const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 mean = *(const float4*)(save + col), invstd = *(const float4*)(save + H + col);
  const float4 gm = *(const float4*)(gamma + col), bt = *(const float4*)(beta + col);
  const float4 al = make_float4(invstd.x * gm.x, invstd.y * gm.y, invstd.z * gm.z, invstd.w * gm.w);
  const float4 bp = make_float4(fmaf(-mean.x, al.x, bt.x), fmaf(-mean.y, al.y, bt.y), fmaf(-mean.z, al.z, bt.z),
                                fmaf(-mean.w, al.w, bt.w));
  // rows past nrows re-read the chunk's last row (never used): branch-free loads, and up to four
  // slabs' loads in flight together
  float4 da[8], y[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int64_t o = (int64_t)(r0 + min(rg + 16 * i, nrows - 1)) * ld + col;
    da[i] = *(const float4*)(dslabs + o);
    y[i] = *(const float4*)(Y + o);
  }
  for (int sl = 1; sl < S; sl += 3) {
    float4 w[3][8];
#pragma unroll
    for (int u = 0; u < 3; ++u)
      if (sl + u < S)
#pragma unroll
        for (int i = 0; i < 8; ++i)
          w[u][i] = *(const float4*)(dslabs + (int64_t)(sl + u) * slab + (int64_t)(r0 + min(rg + 16 * i, nrows - 1)) * ld + col);
#pragma unroll
    for (int u = 0; u < 3; ++u)
      if (sl + u < S)
#pragma unroll
        for (int i = 0; i < 8; ++i) da[i] = f4add(da[i], w[u][i]);
  }
  float4 s1 = zero, s2 = zero;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int rl = rg + 16 * i;
    if (rl < nrows) {
      if (dsum) *(float4*)(dsum + (int64_t)(r0 + rl) * ld + col) = da[i];
      const float d0 = fmaf(y[i].x, al.x, bp.x) > 0.f ? da[i].x : 0.f;
      const float d1 = fmaf(y[i].y, al.y, bp.y) > 0.f ? da[i].y : 0.f;
      const float d2 = fmaf(y[i].z, al.z, bp.z) > 0.f ? da[i].z : 0.f;
      const float d3 = fmaf(y[i].w, al.w, bp.w) > 0.f ? da[i].w : 0.f;
      s1 = f4add(s1, make_float4(d0, d1, d2, d3));
      s2 = make_float4(fmaf(y[i].x - mean.x, d0, s2.x), fmaf(y[i].y - mean.y, d1, s2.y),
                       fmaf(y[i].z - mean.z, d2, s2.z), fmaf(y[i].w - mean.w, d3, s2.w));
    }
  }
  red[0][rg][cg] = s1;
  red[1][rg][cg] = s2;
  __syncthreads();
  if (rg == 0) {
    float4 a = zero, q = zero;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      a = f4add(a, red[0][k][cg]);
      q = f4add(q, red[1][k][cg]);
    }
    float4* o = (float4*)(part + (int64_t)blockIdx.y * H + col);
    o[0] = make_float4(a.x, q.x, a.y, q.y);
    o[1] = make_float4(a.z, q.z, a.w, q.w);
  }
}

// ---------------------------------------------------------------------------------------------
// reparameterization: mu|lv = heads (+bias); z = mu + exp(0.5*lv)*eps; KL partial sums.
// Block: kReparamRows rows (Bp / kReparamRows blocks: the work is latency-bound, so many short
// blocks); each thread's (row, l) elements are loaded before any is used.
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void k_reparam(const float* __restrict__ slabs, int S, int64_t slab, int L,
                                               const float* __restrict__ bmu, const float* __restrict__ blv,
                                               const float* __restrict__ eps, int B, float* __restrict__ HD,
                                               T* __restrict__ Z, int64_t ldz, T* __restrict__ ZT, int64_t ldzt,
                                               float* __restrict__ kl_part) {
  __shared__ float red[4];
  constexpr int PT = kReparamRows * 256 / 256;  // elements per thread at L = 256 (host: L <= 256)
  const int r0 = blockIdx.x * kReparamRows;
  const int ldh = 2 * L, n = kReparamRows * L;
  float mu[PT], lv[PT], e[PT];
#pragma unroll
  for (int j = 0; j < PT; ++j) {
    const int i = threadIdx.x + j * 256, rl = i / L, l = i - rl * L, r = r0 + rl;
    mu[j] = lv[j] = e[j] = 0.f;
    if (i < n && r < B) {
      const int64_t o = (int64_t)r * ldh;
      mu[j] = slabs[o + l];
      lv[j] = slabs[o + L + l];
      for (int z = 1; z < S; ++z) {
        mu[j] += slabs[z * slab + o + l];
        lv[j] += slabs[z * slab + o + L + l];
      }
      e[j] = eps ? eps[(int64_t)r * L + l] : 0.f;
    }
  }
  float kl = 0.f;
#pragma unroll
  for (int j = 0; j < PT; ++j) {
    const int i = threadIdx.x + j * 256, rl = i / L, l = i - rl * L, r = r0 + rl;
    if (i >= n) break;
    float z = 0.f;
    if (r < B) {
      const int64_t o = (int64_t)r * ldh;
      const float m = mu[j] + bmu[l], v = lv[j] + blv[l];
      HD[o + l] = m;
      HD[o + L + l] = v;
      z = m + expf(0.5f * v) * e[j];
      kl += ((1.0f + v) - m * m) - expf(v);
    }
    Z[(int64_t)r * ldz + l] = E<T>::cvt(z);
    if (ZT) ZT[(int64_t)l * ldzt + r] = E<T>::cvt(z);
  }
  kl = wave_sum(kl);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = kl;
  __syncthreads();
  if (threadIdx.x == 0) kl_part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// backward through reparameterization + beta*KL (autograd of model.py:101-103 and
// loss_components.py:77): dmu = dz + beta*mu ; dlv = 0.5*dz*eps*std - 0.5*beta*(1 - exp(lv)).
// dmu_ext / dlv_ext (optional, [B][L]): upstream gradients of mu / logvar from outside the fused
// loss (VAE.forward under torch autograd: gm2_backward_outputs), added to the above.
template <typename T>
__global__ __launch_bounds__(256) void k_reparam_bwd(const float* __restrict__ dz, int S, int64_t slab,
                                                   int64_t ldslab, const float* __restrict__ HD,
                                                   const float* __restrict__ eps, const float* __restrict__ scal,
                                                   int B, int L, T* __restrict__ dH, int64_t ldh,
                                                   const float* __restrict__ dmu_ext,
                                                   const float* __restrict__ dlv_ext, float* __restrict__ colpart) {
  __shared__ float acc[2][256];
  constexpr int PT = kReparamRows;  // elements per thread at L = 256 (host: L <= 256)
  const float beta = scal[kScalBeta];
  const int r0 = blockIdx.x * kReparamRows;
  const int L2 = 2 * L, n = kReparamRows * L;
  // 256 % L == 0 (host-checked): thread t always sees column t % L, so its column sums live in
  // registers and are combined in a fixed order (deterministic bias gradients). Every load of the
  // thread is issued before any is used (the work is latency-bound).
  float dv[PT], muv[PT], lvv[PT], ev[PT];
#pragma unroll
  for (int j = 0; j < PT; ++j) {
    const int i = threadIdx.x + j * 256, rl = i / L, l = i - rl * L, r = r0 + rl;
    dv[j] = muv[j] = lvv[j] = ev[j] = 0.f;
    if (i < n && r < B) {
      const int64_t o = (int64_t)r * ldslab + l;
      dv[j] = dz[o];
      for (int s = 1; s < S; ++s) dv[j] += dz[s * slab + o];
      muv[j] = HD[(int64_t)r * L2 + l];
      lvv[j] = HD[(int64_t)r * L2 + L + l];
      ev[j] = eps[(int64_t)r * L + l];
    }
  }
  float smu = 0.f, slv = 0.f;
#pragma unroll
  for (int j = 0; j < PT; ++j) {
    const int i = threadIdx.x + j * 256, rl = i / L, l = i - rl * L, r = r0 + rl;
    if (i >= n) break;
    float gmu = 0.f, glv = 0.f;
    if (r < B) {
      const float d = dv[j], mu = muv[j], lv = lvv[j], e = ev[j];
      const float sd = expf(0.5f * lv);
      gmu = d + (0.5f * beta) * (2.0f * mu);
      glv = 0.5f * ((d * e) * sd) + (-0.5f * beta + (0.5f * beta) * expf(lv));
      if (dmu_ext) gmu += dmu_ext[(int64_t)r * L + l];
      if (dlv_ext) glv += dlv_ext[(int64_t)r * L + l];
    }
    dH[(int64_t)r * ldh + l] = E<T>::cvt(gmu);
    dH[(int64_t)r * ldh + L + l] = E<T>::cvt(glv);
    smu += gmu;
    slv += glv;
  }
  acc[0][threadIdx.x] = smu;
  acc[1][threadIdx.x] = slv;
  __syncthreads();
  if (threadIdx.x < L) {
    float a = 0.f, b = 0.f;
    for (int k = threadIdx.x; k < 256; k += L) { a += acc[0][k]; b += acc[1][k]; }
    colpart[(int64_t)blockIdx.x * L2 + threadIdx.x] = a;
    colpart[(int64_t)blockIdx.x * L2 + L + threadIdx.x] = b;
  }
}

// z = mu + exp(0.5*lv)*eps (model.py:100-104 VAE.reparameterization with the noise given),
// and its backward (mode 1): dmu = dz, dlv = 0.5*dz*eps*exp(0.5*lv). Elementwise over n*L.
__global__ __launch_bounds__(256) void k_reparameterize(int64_t n, const float* __restrict__ mu,
                                                      const float* __restrict__ lv, const float* __restrict__ eps,
                                                      float* __restrict__ z, const float* __restrict__ dz,
                                                      float* __restrict__ dmu, float* __restrict__ dlv) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float sd = expf(0.5f * lv[i]);
    if (z) z[i] = mu[i] + sd * eps[i];
    if (dz) {
      const float d = dz[i];
      dmu[i] = d;
      dlv[i] = 0.5f * ((d * eps[i]) * sd);
    }
  }
}

// dL/dlogit of the output layer from an upstream dL/dp (autograd of torch.sigmoid, model.py:90):
// dl = dp * (1 - p) * p, written as T [Bp][ldd] (rows >= B and columns >= G zero) with per-(64-row
// chunk, column) partial sums for the output bias gradient. Block: 256 columns x 64 rows.
template <typename T>
__global__ __launch_bounds__(256) void k_sigmoid_bwd(const float* __restrict__ p, const float* __restrict__ dp,
                                                   int64_t ldp, int B, int G, int Gp, T* __restrict__ dL,
                                                   int64_t ldd, float* __restrict__ colpart) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int r0 = blockIdx.y * 64;
  if (c >= Gp) return;
  float cs = 0.f;
  for (int rl = 0; rl < 64; ++rl) {
    const int r = r0 + rl;
    float dl = 0.f;
    if (r < B && c < G) {
      const float pv = p[(int64_t)r * ldp + c];
      dl = (dp[(int64_t)r * ldp + c] * (1.0f - pv)) * pv;
    }
    cs += dl;
    dL[(int64_t)r * ldd + c] = E<T>::cvt(dl);
  }
  colpart[(int64_t)blockIdx.y * Gp + c] = cs;
}

// The forward's tail in one launch: block 0 = loss slots [0], [1] (sum of the output-layer tile
// partials) and [2] (KL partials), fp64 per-thread strided sums + wave sums; blocks 1.. = the
// output-layer bias gradient column sums in k_colsum2's order (rows = strain tiles).
__global__ __launch_bounds__(256) void k_fwd_tail(const float* __restrict__ lpart, int nl, const float* __restrict__ kpart,
                                                int nk, double* __restrict__ loss, const float* __restrict__ cpart,
                                                int rows, int64_t ld, int64_t n, float* __restrict__ cout,
                                                int* __restrict__ hdr, int hv0, int hv1) {
  __shared__ double red[4];
  __shared__ float redf[4][64];
  if (blockIdx.x == 0) {
    if (hdr && threadIdx.x == 0) {
      hdr[0] = hv0;
      hdr[1] = hv1;
    }
    for (int k = 0; k < 3; ++k) {
      const float* part = k < 2 ? lpart + k : kpart;
      const int cnt = k < 2 ? nl : nk, stride = k < 2 ? 2 : 1;
      double s = 0.0;
      for (int b = threadIdx.x; b < cnt; b += 256 * 8) {  // loads 8 at a time, added in order
        float q[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) q[j] = b + 256 * j < cnt ? part[(int64_t)(b + 256 * j) * stride] : 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (b + 256 * j < cnt) s += (double)q[j];
      }
      s = wave_sum_d(s);
      if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
      __syncthreads();
      if (threadIdx.x == 0) loss[k] = red[0] + red[1] + red[2] + red[3];
      __syncthreads();
    }
    return;
  }
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int64_t c = (int64_t)(blockIdx.x - 1) * 64 + cl;
  float sum = 0.f;
  if (c < n)
    for (int r = rg; r < rows; r += 4) sum += cpart[(int64_t)r * ld + c];
  redf[rg][cl] = sum;
  __syncthreads();
  if (rg == 0 && c < n) cout[c] = (redf[0][cl] + redf[1][cl]) + (redf[2][cl] + redf[3][cl]);
}

// ---------------------------------------------------------------------------------------------
// GEMM shadows: padded (and transposed) T copies of the Linear weights. Tile 64x64.
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void k_shadow_sync(TensorTable tt, const float* __restrict__ params) {
  __shared__ float tile[64][65];
  int ti = 0;
  while (ti + 1 < tt.n && (int64_t)blockIdx.x >= tt.t[ti + 1].tile0) ++ti;
  const TensorDesc& d = tt.t[ti];
  const int64_t local = blockIdx.x - d.tile0;
  const int64_t tcols = (d.cols + 63) / 64;
  const int64_t r0 = (local / tcols) * 64, c0 = (local % tcols) * 64;
  const float* src = params + d.off;
  T* sh = (T*)d.shadow;
  T* shT = (T*)d.shadowT;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int rl = i >> 6, cl = i & 63;
    const int64_t r = r0 + rl, c = c0 + cl;
    float v = 0.f;
    if (r < d.rows && c < d.cols) {
      v = src[r * d.cols + c];
      if (sh) sh[(d.srow0 + r) * d.sld + c] = E<T>::cvt(v);
    }
    tile[cl][rl] = v;
  }
  __syncthreads();
  if (shT) {
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
      const int cl = i >> 6, rl = i & 63;
      const int64_t r = r0 + rl, c = c0 + cl;
      if (r < d.rows && c < d.cols) shT[c * d.tld + d.srow0 + r] = E<T>::cvt(tile[cl][rl]);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// clip_grad_norm_ statistics (+ L1 term) and the fused L1 + clip + Adam update
// ---------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void store4(T* dst, float a, float b, float c, float d) {
  if constexpr (sizeof(T) == 2) {
    uint2 pk;
    pk.x = f2bf2(a, b);
    pk.y = f2bf2(c, d);
    *(uint2*)dst = pk;
  } else {
    *(float4*)dst = make_float4(a, b, c, d);
  }
}

__device__ __forceinline__ float sgnf(float x) { return (float)((x > 0.f) - (x < 0.f)); }

// 16-byte non-temporal (streaming) load / store: for data every pass touches exactly once
// (measured on the Adam pass: 650 -> 546 us, 5.4 -> 6.45 TB/s)
__device__ __forceinline__ float4 ntload4(const float* p) {
  const f32x4 v = __builtin_nontemporal_load((const f32x4*)p);
  return make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void ntstore4(float* p, const float (&v)[4]) {
  __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, (f32x4*)p);
}

// sum of g[i]^2 over [a, b), grid-stride (16-B loads between the scalar head and tail)
__device__ __forceinline__ double seg_sumsq(const float* __restrict__ g, int64_t a, int64_t b) {
  double ss = 0.0;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x, stride = (int64_t)gridDim.x * 256;
  if (a >= b) return ss;
  const int64_t va = (a + 3) & ~(int64_t)3, vb = b & ~(int64_t)3;
  if (va >= vb) {
    for (int64_t i = a + t; i < b; i += stride) ss += (double)g[i] * g[i];
    return ss;
  }
  for (int64_t i = va / 4 + t; i < vb / 4; i += stride) {
    const float4 gv = ntload4(g + 4 * i);
    ss += (double)gv.x * gv.x + (double)gv.y * gv.y + (double)gv.z * gv.z + (double)gv.w * gv.w;
  }
  if (t < va - a) ss += (double)g[a + t] * g[a + t];
  if (t < b - vb) ss += (double)g[vb + t] * g[vb + t];
  return ss;
}

// the GEMM-epilogue statistics are used when the caller vouches for them (scal[kScalNormAhead]),
// the last training call recorded them (hdr[0]) and there is no L1 term (which needs sign(theta))
__device__ __forceinline__ bool use_ahead(const NormAhead& na, const float* scal) {
  return na.hdr && scal[kScalNormAhead] != 0.f && scal[kScalLambda] == 0.f && na.hdr[0] != 0;
}

__global__ __launch_bounds__(256) void k_grad_stats(const float* __restrict__ p, const float* __restrict__ g,
                                                  int64_t n, const float* __restrict__ scal,
                                                  double* __restrict__ part, NormAhead na) {
  __shared__ double red[2][4];
  const float lam = scal[kScalLambda];
  double ss = 0.0, ab = 0.0;
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * 256;
  if (lam != 0.f) {  // L1 present: the norm needs sign(p), the loss needs sum|p|
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
      const float4 pv = ntload4(p + 4 * i), gv = ntload4(g + 4 * i);
      const float a = gv.x + lam * sgnf(pv.x), b = gv.y + lam * sgnf(pv.y);
      const float c = gv.z + lam * sgnf(pv.z), d = gv.w + lam * sgnf(pv.w);
      ss += (double)a * a + (double)b * b + (double)c * c + (double)d * d;
      ab += (double)fabsf(pv.x) + (double)fabsf(pv.y) + (double)fabsf(pv.z) + (double)fabsf(pv.w);
    }
    for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
      const float a = g[i] + lam * sgnf(p[i]);
      ss += (double)a * a;
      ab += fabs((double)p[i]);
    }
  } else if (use_ahead(na, scal)) {  // the two big weight gradients were summed as they were written
    ss = seg_sumsq(g, 0, na.lo0) + seg_sumsq(g, na.hi0, na.lo9) + seg_sumsq(g, na.hi9, n);
  } else {  // no L1 term (v0): gradients only, half the traffic
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
      const float4 gv = ntload4(g + 4 * i);
      ss += (double)gv.x * gv.x + (double)gv.y * gv.y + (double)gv.z * gv.z + (double)gv.w * gv.w;
    }
    for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
      ss += (double)g[i] * g[i];
  }
  ss = wave_sum_d(ss);
  ab = wave_sum_d(ab);
  if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = ss; red[1][threadIdx.x >> 6] = ab; }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[blockIdx.x * 2 + 0] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    part[blockIdx.x * 2 + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

__global__ __launch_bounds__(256) void k_grad_finalize(const double* __restrict__ part, int nb,
                                                     const float* __restrict__ scal, float* __restrict__ clip,
                                                     double* __restrict__ l1abs, NormAhead na) {
  __shared__ double red[2][4];
  double ss = 0.0, ab = 0.0;
  // (each thread's strided terms are loaded 8 at a time before they are added, in the same order:
  // one workgroup, so the latency of dependent loads would be the kernel's whole time)
  for (int b = threadIdx.x; b < nb; b += 256 * 8) {
    double qs[8], qa[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = b + 256 * j;
      qs[j] = i < nb ? part[2 * i] : 0.0;
      qa[j] = i < nb ? part[2 * i + 1] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (b + 256 * j < nb) { ss += qs[j]; ab += qa[j]; }
  }
  if (use_ahead(na, scal)) {
    const int cnt = na.hdr[1];
    for (int b = threadIdx.x; b < cnt; b += 256 * 8) {
      double q[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) q[j] = b + 256 * j < cnt ? na.sq[b + 256 * j] : 0.0;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (b + 256 * j < cnt) ss += q[j];
    }
  }
  ss = wave_sum_d(ss);
  ab = wave_sum_d(ab);
  if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = ss; red[1][threadIdx.x >> 6] = ab; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double s = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    const float norm = (float)sqrt(s);
    const float mx = scal[kScalMaxNorm];
    float c = 1.0f;
    if (mx > 0.f) c = fminf(mx / (norm + 1e-6f), 1.0f);
    clip[0] = c;
    clip[1] = norm;
    if (l1abs) {  // loss record slots 3 (sum |theta|) and 4 (the norm)
      l1abs[0] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
      l1abs[1] = (double)norm;
    }
  }
}

// fused L1 + clip + Adam over one tensor table entry per block group, writing the fp32 master and
// the natural-layout GEMM shadow in the same pass (30 B/param of HBM traffic instead of 30 + 6)
// (one 4096-element block `blk` of tensor d)
template <typename T>
__device__ __forceinline__ void adam_block(const TensorDesc& d, int64_t blk, const float* __restrict__ g,
                                           float* __restrict__ p, float* __restrict__ m, float* __restrict__ v,
                                           const float* __restrict__ scal, const float* __restrict__ clip) {
  const int64_t numel = d.rows * d.cols;
  const int64_t e0 = (blk - d.tile0) * 4096;  // 4096 elements per block
  const float lam = scal[kScalLambda], negstep = scal[kScalNegStep], bc2s = scal[kScalBc2Sqrt];
  const float w1 = scal[kScalOneMinusB1], b2 = scal[kScalBeta2], w2 = scal[kScalOneMinusB2];
  const float aeps = scal[kScalAdamEps];
  const float cc = clip[0];
  T* sh = (T*)d.shadow;
  if (e0 + 4096 <= numel) {
    // whole block: all 16 loads of the thread in flight before the first update; every byte is
    // touched once per step, so loads and stores are non-temporal (streamed past the caches)
    float4 pv[4], gv[4], mv[4], vv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t gi = d.off + e0 + (int64_t)(k * 256 + threadIdx.x) * 4;
      pv[k] = ntload4(p + gi);
      gv[k] = ntload4(g + gi);
      mv[k] = ntload4(m + gi);
      vv[k] = ntload4(v + gi);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t e = e0 + (int64_t)(k * 256 + threadIdx.x) * 4;
      const int64_t gi = d.off + e;
      float pe[4] = {pv[k].x, pv[k].y, pv[k].z, pv[k].w}, ge[4] = {gv[k].x, gv[k].y, gv[k].z, gv[k].w};
      float me[4] = {mv[k].x, mv[k].y, mv[k].z, mv[k].w}, ve[4] = {vv[k].x, vv[k].y, vv[k].z, vv[k].w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float gg = (ge[u] + lam * sgnf(pe[u])) * cc;
        me[u] = me[u] + w1 * (gg - me[u]);
        ve[u] = ve[u] * b2;
        ve[u] = ve[u] + w2 * gg * gg;
        const float denom = sqrtf(ve[u]) / bc2s + aeps;
        pe[u] = pe[u] + negstep * (me[u] / denom);
      }
      ntstore4(p + gi, pe);
      ntstore4(m + gi, me);
      ntstore4(v + gi, ve);
      if (sh) {
        int64_t r = e / d.cols, c = e - r * d.cols;
        if ((d.cols & 3) == 0 && (d.sld & 3) == 0) {
          store4<T>(sh + (d.srow0 + r) * d.sld + c, pe[0], pe[1], pe[2], pe[3]);
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            sh[(d.srow0 + r) * d.sld + c] = E<T>::cvt(pe[u]);
            if (++c == d.cols) { c = 0; ++r; }
          }
        }
      }
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t e = e0 + (int64_t)(k * 256 + threadIdx.x) * 4;  // 4 consecutive elements
    if (e >= numel) break;
    const int64_t gi = d.off + e;
    float4 pv, gv, mv, vv;
    const bool full = e + 4 <= numel;
    if (full) {
      pv = *(const float4*)(p + gi);
      gv = *(const float4*)(g + gi);
      mv = *(const float4*)(m + gi);
      vv = *(const float4*)(v + gi);
    } else {
      float* a[4] = {&pv.x, &pv.y, &pv.z, &pv.w};
      float* b[4] = {&gv.x, &gv.y, &gv.z, &gv.w};
      float* c[4] = {&mv.x, &mv.y, &mv.z, &mv.w};
      float* dd[4] = {&vv.x, &vv.y, &vv.z, &vv.w};
      for (int u = 0; u < 4; ++u) {
        const bool ok = e + u < numel;
        *a[u] = ok ? p[gi + u] : 0.f;
        *b[u] = ok ? g[gi + u] : 0.f;
        *c[u] = ok ? m[gi + u] : 0.f;
        *dd[u] = ok ? v[gi + u] : 0.f;
      }
    }
    float pe[4] = {pv.x, pv.y, pv.z, pv.w}, ge[4] = {gv.x, gv.y, gv.z, gv.w};
    float me[4] = {mv.x, mv.y, mv.z, mv.w}, ve[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float gg = (ge[u] + lam * sgnf(pe[u])) * cc;
      me[u] = me[u] + w1 * (gg - me[u]);           // exp_avg.lerp_(grad, 1 - beta1)
      ve[u] = ve[u] * b2;
      ve[u] = ve[u] + w2 * gg * gg;                // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
      const float denom = sqrtf(ve[u]) / bc2s + aeps;
      pe[u] = pe[u] + negstep * (me[u] / denom);   // param.addcdiv_(exp_avg, denom, -step_size)
    }
    if (full) {
      *(float4*)(p + gi) = make_float4(pe[0], pe[1], pe[2], pe[3]);
      *(float4*)(m + gi) = make_float4(me[0], me[1], me[2], me[3]);
      *(float4*)(v + gi) = make_float4(ve[0], ve[1], ve[2], ve[3]);
    } else {
      for (int u = 0; u < 4; ++u)
        if (e + u < numel) { p[gi + u] = pe[u]; m[gi + u] = me[u]; v[gi + u] = ve[u]; }
    }
    if (sh) {
      int64_t r = e / d.cols, c = e - r * d.cols;
      if (full && (d.cols & 3) == 0 && (d.sld & 3) == 0) {  // 4 elements of one row: one 8/16-B store
        store4<T>(sh + (d.srow0 + r) * d.sld + c, pe[0], pe[1], pe[2], pe[3]);
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (e + u < numel) sh[(d.srow0 + r) * d.sld + c] = E<T>::cvt(pe[u]);
          if (++c == d.cols) { c = 0; ++r; }
        }
      }
    }
  }
}

// blocks blockIdx.x, + gridDim.x, ... of the table (one per workgroup unless the grid is capped:
// the deferred output-layer update runs on a few workgroups per CU beside the hidden layers)
template <typename T>
__global__ __launch_bounds__(256) void k_adam_fused(TensorTable tt, const float* __restrict__ g, float* __restrict__ p,
                                                  float* __restrict__ m, float* __restrict__ v,
                                                  const float* __restrict__ scal, const float* __restrict__ clip,
                                                  int64_t nblocks, float* __restrict__ scal_copy) {
  // (a copy of the scalar block for a queued update that runs after the caller's block is gone)
  if (scal_copy && blockIdx.x == 0 && threadIdx.x < kNumScal) scal_copy[threadIdx.x] = scal[threadIdx.x];
  int ti = 0;
  for (int64_t blk = blockIdx.x; blk < nblocks; blk += gridDim.x) {
    while (ti + 1 < tt.n && blk >= tt.t[ti + 1].tile0) ++ti;
    adam_block<T>(tt.t[ti], blk, g, p, m, v, scal, clip);
  }
}

// C (row-split into C0/C1) = sum of S fp32 split-K slabs [S][M][N] (fixed order: deterministic)
__global__ __launch_bounds__(256) void k_slab_sum(const float* __restrict__ slabs, int S, int64_t slab, int M, int N,
                                                float* __restrict__ C0, float* __restrict__ C1, int msplit,
                                                int64_t ldc) {
  const int64_t total = (int64_t)M * N;
  // rows of C are 16-B aligned and N % 4 == 0: the 4 elements of a thread are one row's float4
  const bool vec = (N & 3) == 0 && (ldc & 3) == 0 && ((((uintptr_t)C0) | ((uintptr_t)C1)) & 15) == 0;
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < total; i += (int64_t)gridDim.x * 1024) {
    float4 a = *(const float4*)(slabs + i);
    if (S <= 8) {  // every slab's load in flight, summed in slab order
      float4 b[7];
#pragma unroll
      for (int s = 1; s < 8; ++s)
        if (s < S) b[s - 1] = *(const float4*)(slabs + s * slab + i);
#pragma unroll
      for (int s = 1; s < 8; ++s)
        if (s < S) { a.x += b[s - 1].x; a.y += b[s - 1].y; a.z += b[s - 1].z; a.w += b[s - 1].w; }
    } else {
      for (int s = 1; s < S; ++s) {
        const float4 b = *(const float4*)(slabs + s * slab + i);
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      }
    }
    if (vec && i + 3 < total) {
      const int m = (int)(i / N), n = (int)(i - (int64_t)m * N);
      float* dst = m < msplit ? C0 + (int64_t)m * ldc + n : C1 + (int64_t)(m - msplit) * ldc + n;
      *(float4*)dst = a;
      continue;
    }
    const float e[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t k = i + u;
      if (k >= total) break;
      const int m = (int)(k / N), n = (int)(k - (int64_t)m * N);
      if (m < msplit) C0[(int64_t)m * ldc + n] = e[u];
      else C1[(int64_t)(m - msplit) * ldc + n] = e[u];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// BatchNorm finalize + apply in one launch per layer and direction. Every block first turns the
// chunk partials of its 256 columns into the layer's coefficients (the fp64 chunk merge, ~32
// L2-resident float2 per column, recomputed identically by each row block) and keeps them in LDS;
// row block 0 owns the per-column side outputs (save, running statistics, dgamma / dbeta).
// Then a vectorised elementwise pass over 64 rows x 256 columns (4 columns per thread).
// ---------------------------------------------------------------------------------------------
// forward coefficients (alpha = invstd*gamma, beta' = fma(-mean, alpha, beta)) of column `col`
// (SyncBN: `sync` holds the all-reduced [sum y | sum y^2 | rows] of every rank's batch, fp64; the
// statistics are then the global batch's, N = sync[2H] rows)
__device__ __forceinline__ void bn_sync_stats(const double* __restrict__ sync, int H, int col, double& mean,
                                              double& var, double& n) {
  n = sync[2 * H];
  mean = sync[col] / n;
  var = fmax(sync[H + col] / n - mean * mean, 0.0);
}

__device__ __forceinline__ float2 bn_fwd_coef(const float2* __restrict__ part, int B, int H, int train,
                                     const float* __restrict__ gamma, const float* __restrict__ beta, float* rmean,
                                     float* rvar, float* save, int col, bool own, const double* __restrict__ sync) {
  float invstd, meanf;
  if (train) {
    double mean, var, n = (double)B;
    if (sync) bn_sync_stats(sync, H, col, mean, var, n);
    else bn_merge(part, B, H, col, mean, var);
    return bn_fwd_train_coef(mean, var, n, H, col, gamma, beta, rmean, rvar, save, own);
  } else {
    // eval transform bit-identical to the reference CPU path (pinned in tests): float
    // invstd = 1/sqrt(rv + eps), alpha = gamma*invstd, beta' = fma(-mean, alpha, beta)
    meanf = rmean[col];
    invstd = 1.0f / sqrtf(rvar[col] + (float)kBnEps);
    if (own && save) {
      save[col] = meanf;
      save[H + col] = invstd;
    }
  }
  const float alpha = invstd * gamma[col];
  return make_float2(alpha, fmaf(-meanf, alpha, beta[col]));
}

// A = relu(y*alpha + beta') for rows < B, 0 for rows in [B, Bp). Grid: (ceil(H/256), Bp/64).
template <typename T>
__global__ __launch_bounds__(256) void k_bn_fwd_apply(const float* __restrict__ Y, int64_t ld,
                                                    const float2* __restrict__ part, int B, int H, int train,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    float* rmean, float* rvar, float* save, T* __restrict__ A,
                                                    const double* __restrict__ sync) {
  __shared__ float2 cf[256];
  const int c0 = blockIdx.x * 256;
  const int cl = (threadIdx.x & 63) * 4, rg = threadIdx.x >> 6;
  const int c = c0 + cl;
  const int r0 = blockIdx.y * 64;
  if (c0 + (int)threadIdx.x < H)
    cf[threadIdx.x] = bn_fwd_coef(part, B, H, train, gamma, beta, rmean, rvar, save, c0 + threadIdx.x,
                                  blockIdx.y == 0, sync);
  __syncthreads();
  if (c >= H) return;  // H % 128 == 0: the last block may cover only 128 of its 256 columns
  const float2 k0 = cf[cl], k1 = cf[cl + 1], k2 = cf[cl + 2], k3 = cf[cl + 3];
  float4 y[16];  // all 16 rows of this thread in flight at once (rows >= B re-read row B-1, unused)
#pragma unroll
  for (int i = 0; i < 16; ++i) y[i] = *(const float4*)(Y + (int64_t)min(r0 + rg + 4 * i, B - 1) * ld + c);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int r = r0 + rg + 4 * i;
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < B) {
      o.x = fmaxf(fmaf(y[i].x, k0.x, k0.y), 0.f);
      o.y = fmaxf(fmaf(y[i].y, k1.x, k1.y), 0.f);
      o.z = fmaxf(fmaf(y[i].z, k2.x, k2.y), 0.f);
      o.w = fmaxf(fmaf(y[i].w, k3.x, k3.y), 0.f);
    }
    store4<T>(A + (int64_t)r * ld + c, o.x, o.y, o.z, o.w);
  }
}

// dx = (do - grad_mean - (y-mean)*proj_scale) * alpha, do = da*[y*alpha+beta' > 0]; rows >= B -> 0;
// grad_mean = sum(do)/B, proj_scale = sum((y-mean)do)*invstd^2/B in train mode; in eval mode
// BatchNorm is the affine map y -> (y - rm)*invstd*gamma + beta and both are 0 (no batch
// coupling). dgamma = sum((y-mean)do)*invstd, dbeta = sum(do) from the chunk partials (fp64).
// Per-(64-row chunk, column) sums of dx -> colpart (the pre-BN Linear bias gradient; summed by
// k_colsum2 -- an in-launch last-arriver sum measured +30 us per launch on this shape).
template <typename T>
__global__ __launch_bounds__(256) void k_bn_bwd_apply(const float* __restrict__ da, const float* __restrict__ Y,
                                                    int64_t ld, const float2* __restrict__ part, int B, int H,
                                                    int train, const float* __restrict__ save,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                    T* __restrict__ dY, float* __restrict__ colpart,
                                                    const double* __restrict__ sync, T* __restrict__ dYT,
                                                    int64_t ldt) {
  __shared__ float4 cf4[5][64];  // [mean, alpha, beta', grad_mean, proj_scale][column / 4]
  __shared__ float4 red[4][64];
  // dYT (bf16 only): the output written transposed, dYT [H][ldt] (the input layer's K-major
  // weight-gradient operand), instead of dY: each thread then takes 16 CONSECUTIVE rows
  // (rg * 16 + i instead of rg + 4 i), so each of its 4 columns leaves as two 16-B row runs of dYT
  // (no LDS: the launch keeps room beside a co-running GEMM workgroup)
  const bool blk = sizeof(T) == 2 && dYT != nullptr;
  float* cf = (float*)cf4;
  const int c0 = blockIdx.x * 256;
  const int cg = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = c0 + cg * 4;
  const int r0 = blockIdx.y * 64;
  const bool ok = c < H;
  {
    const int t = threadIdx.x, col = c0 + t;
    if (col < H) {
      double s1, s2;
      bn_bwd_sums_ld([&](int ch) { return part[(int64_t)ch * H + col]; }, B, s1, s2);
      const float invstd = save[H + col];
      if (blockIdx.y == 0) {
        dgamma[col] = (float)(s2 * invstd);
        dbeta[col] = (float)s1;
      }
      // (SyncBN: the coupling terms use the global batch's sums; dgamma / dbeta above stay this
      // rank's share, which the gradient all-reduce sums)
      const double g1 = sync ? sync[col] : s1, g2 = sync ? sync[H + col] : s2, nb = sync ? sync[2 * H] : (double)B;
      float c5[5];
      bn_bwd_coef(g1, g2, nb, train, H, col, save, gamma, beta, c5);
#pragma unroll
      for (int k = 0; k < 5; ++k) cf[256 * k + t] = c5[k];
    }
  }
  __syncthreads();
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok) {
    // all 16 rows of dA and Y of this thread in flight at once
    float4 av[16], yv[16];  // (rows >= B re-read row B-1, unused)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int64_t o = (int64_t)min(r0 + (blk ? rg * 16 + i : rg + 4 * i), B - 1) * ld + c;
      av[i] = *(const float4*)(da + o);
      yv[i] = *(const float4*)(Y + o);
    }
    const float4 mean = cf4[0][cg], al = cf4[1][cg], be = cf4[2][cg], gm = cf4[3][cg], ps = cf4[4][cg];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int r = r0 + (blk ? rg * 16 + i : rg + 4 * i);
      float4 dx = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < B) {
        const float4 a = av[i];
        const float4 y = yv[i];
        const float d0 = fmaf(y.x, al.x, be.x) > 0.f ? a.x : 0.f;
        const float d1 = fmaf(y.y, al.y, be.y) > 0.f ? a.y : 0.f;
        const float d2 = fmaf(y.z, al.z, be.z) > 0.f ? a.z : 0.f;
        const float d3 = fmaf(y.w, al.w, be.w) > 0.f ? a.w : 0.f;
        dx.x = (d0 - gm.x - (y.x - mean.x) * ps.x) * al.x;
        dx.y = (d1 - gm.y - (y.y - mean.y) * ps.y) * al.y;
        dx.z = (d2 - gm.z - (y.z - mean.z) * ps.z) * al.z;
        dx.w = (d3 - gm.w - (y.w - mean.w) * ps.w) * al.w;
      }
      acc.x += dx.x; acc.y += dx.y; acc.z += dx.z; acc.w += dx.w;
      if (blk) {
        av[i] = dx;  // (kept for the transposed stores below)
        continue;
      }
      store4<T>(dY + (int64_t)r * ld + c, dx.x, dx.y, dx.z, dx.w);
    }
    if constexpr (sizeof(T) == 2) {
      if (blk) {  // column c + u: rows r0 + rg*16 .. +15 as two 16-B runs
        T* dst = dYT + (int64_t)c * ldt + r0 + rg * 16;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            float e[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float4 v = av[h * 8 + j];
              e[j] = u == 0 ? v.x : u == 1 ? v.y : u == 2 ? v.z : v.w;
            }
            uint4 pk;
            pk.x = f2bf2(e[0], e[1]);
            pk.y = f2bf2(e[2], e[3]);
            pk.z = f2bf2(e[4], e[5]);
            pk.w = f2bf2(e[6], e[7]);
            *(uint4*)(dst + (int64_t)u * ldt + h * 8) = pk;
          }
        }
      }
    }
  }
  red[rg][cg] = acc;
  __syncthreads();
  if (rg == 0 && ok) {
    float4 v = red[0][cg];
    for (int k = 1; k < 4; ++k) { v.x += red[k][cg].x; v.y += red[k][cg].y; v.z += red[k][cg].z; v.w += red[k][cg].w; }
    *(float4*)(colpart + (int64_t)blockIdx.y * H + c) = v;
  }
}

// SyncBN: this rank's per-column sums of the batch, from the chunk partials, for the all-reduce:
//   forward  (mode 0): out = [sum y | sum y^2 | rows, 0]  (from the chunk (mean, M2) pairs)
//   backward (mode 1): out = [sum do | sum (y - mean) do | rows, 0]
// fp64 throughout (sum y^2 - N mean^2 keeps ~1e-16 * (mean / std)^2 relative error in the variance)
__global__ __launch_bounds__(256) void k_bn_sync_pack(const float2* __restrict__ part, int B, int H, int mode,
                                                    double* __restrict__ out) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col == 0) {
    out[2 * H] = (double)B;
    out[2 * H + 1] = 0.0;
  }
  if (col >= H) return;
  const int nch = (B + kBnRowChunk - 1) / kBnRowChunk;
  double a = 0.0, b = 0.0;
  for (int ch = 0; ch < nch; ++ch) {
    const float2 p = part[(int64_t)ch * H + col];
    if (mode == 0) {
      const double nb = (double)min(kBnRowChunk, B - ch * kBnRowChunk), m = (double)p.x;
      a += nb * m;
      b += (double)p.y + nb * m * m;
    } else {
      a += (double)p.x;
      b += (double)p.y;
    }
  }
  out[col] = a;
  out[H + col] = b;
}

// SyncBN on a rank with no rows this step: the running statistics still follow the global batch
// (the same update every rank applies in k_bn_fwd_apply)
__global__ __launch_bounds__(256) void k_bn_sync_running(const double* __restrict__ sync, int H, float* rmean,
                                                       float* rvar) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= H) return;
  double mean, var, n;
  bn_sync_stats(sync, H, col, mean, var, n);
  const double unb = n > 1.0 ? var * n / (n - 1.0) : var;
  rmean[col] = (float)(kBnMomentum * mean + (1.0 - kBnMomentum) * (double)rmean[col]);
  rvar[col] = (float)(kBnMomentum * unb + (1.0 - kBnMomentum) * (double)rvar[col]);
}

// dst[c][r] = src[r][c] over an R x Cn block (both multiples of 64): 64 x 64 tiles through LDS,
// 16-byte loads and stores (each output row segment = 64 contiguous elements). Used for the small
// activations whose transposed copy turns a weight-gradient GEMM's MN-major operand K-major.
// ---------------------------------------------------------------------------------------------
// bf16x3 split of fp32 rows for the sampling decode's output layer (decode_chain, GM2_OPT_SAMPLE_SPLIT):
// x = hi + lo + r with hi = bf16(x), lo = bf16(x - hi) (x - hi is exact in fp32), |r| <= 2^-16 |x|.
// Row r of X [rows][ldx] (K columns, K % 32 == 0) -> out [r][2K], interleaved per 32 columns: the
// 64-column K-tile c of out holds hi[32c .. 32c+32) then lo[32c .. 32c+32). The decode's
// activations and output weights both take this layout, and the GEMM's main loop (mainloop_pp, S3)
// multiplies each K-tile's halves as hi.hi + hi.lo + lo.hi -- the fp32 product up to 3.02 x 2^-16
// |x| |w| per term -- from 2K columns of operand bytes instead of the 3K of a (hi|hi|lo).(hi|lo|hi)
// concatenation. Rows in [rows, rows_pad) are zero. Per row r it also writes rn[r] = ||x_r||_2 (0 for
// pad rows) -- the per-element error bounds of the decode's band check (MaskOut::rn / cn) -- and the
// block maximum of those norms over each 256-row block b into blk[b] (fp32 bits, non-negative floats
// order as unsigned) by one atomic max per workgroup: the per-tile gate (MaskGate) of the split output
// layer. Each workgroup takes 16 consecutive rows (one wave 4), so it touches one block word only.
// (The first form kept ONE global maximum with one atomic per row into a single word: the launches ran
// at that word's atomic rate, 65,536 rows in 750 us.)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_split3(const float* __restrict__ X, int64_t ldx, int rows, int K,
                                              bf16_t* __restrict__ out, int64_t ldo, float* __restrict__ rn,
                                              unsigned* __restrict__ blk, bf16_t* __restrict__ out1) {
  __shared__ float wmax[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float mx = 0.f;
#pragma unroll 1
  for (int q = 0; q < 4; ++q) {
    const int r = blockIdx.x * 16 + wv * 4 + q;
    float ss = 0.f;
    for (int k0 = lane * 8; k0 < K; k0 += 512) {
      float x[8];
      if (r < rows) {
        const float4 a = *(const float4*)(X + (int64_t)r * ldx + k0), b = *(const float4*)(X + (int64_t)r * ldx + k0 + 4);
        x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = 0.f;
      }
      uint32_t hw[4], lw[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float h0 = bf2f(f2bf(x[2 * e])), h1 = bf2f(f2bf(x[2 * e + 1]));
        hw[e] = f2bf2(x[2 * e], x[2 * e + 1]);
        lw[e] = f2bf2(x[2 * e] - h0, x[2 * e + 1] - h1);
        ss = fmaf(x[2 * e], x[2 * e], ss);
        ss = fmaf(x[2 * e + 1], x[2 * e + 1], ss);
      }
      const uint4 hv = make_uint4(hw[0], hw[1], hw[2], hw[3]), lv = make_uint4(lw[0], lw[1], lw[2], lw[3]);
      bf16_t* o = out + (int64_t)r * ldo + 2 * (k0 & ~31) + (k0 & 31);
      *(uint4*)(o) = hv;
      *(uint4*)(o + 32) = lv;
      if (out1) *(uint4*)(out1 + (int64_t)r * K + k0) = hv;  // (the single-product tier's operand: hi only)
    }
    // (the bound uses the norm rounded up: sqrt of a sum of squares carried in fp32 is within a few
    // ulps of the true norm; x 1.0001 covers that with room)
    const float nrm = r < rows ? sqrtf(wave_sum(ss)) * 1.0001f : 0.f;
    if (lane == 0) rn[r] = nrm;
    mx = fmaxf(mx, nrm);
  }
  if (lane == 0) wmax[wv] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float m = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
    atomicMax(blk + blockIdx.x / 16, __float_as_uint(m));
  }
}

// ---------------------------------------------------------------------------------------------
// bf16 gradient exchange (gm2/ddp.py bf16_exchange_sum, gm2.h gm2_exchange_*): pack rounds the fp32
// gradient to bf16 (RNE, zero pad up to n_pad), ranksum forms out[i] = bf16(((p_0[i] + p_1[i]) + ...)
// + p_{world-1}[i]) in fp32 in rank order from the world's received bf16 chunks, unpack widens the
// gathered bf16 vector back into the fp32 gradient. 8 elements per thread (16-B bf16 / 32-B fp32).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_exchange_pack(const float* __restrict__ x, int64_t n, bf16_t* __restrict__ out,
                                                     int64_t n_pad) {
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8; i < n_pad; i += (int64_t)gridDim.x * 256 * 8) {
    uint32_t w[4];
    if (i + 8 <= n && (((uintptr_t)(x + i)) & 15) == 0) {
      const float4 a = *(const float4*)(x + i), b = *(const float4*)(x + i + 4);
      w[0] = f2bf2(a.x, a.y); w[1] = f2bf2(a.z, a.w); w[2] = f2bf2(b.x, b.y); w[3] = f2bf2(b.z, b.w);
    } else {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = i + e < n ? x[i + e] : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = f2bf2(v[2 * e], v[2 * e + 1]);
    }
    if (i + 8 <= n_pad) {
      *(uint4*)(out + i) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (i + e < n_pad) out[i + e] = (bf16_t)(w[e >> 1] >> (16 * (e & 1)));
    }
  }
}

__global__ __launch_bounds__(256) void k_exchange_ranksum(const bf16_t* __restrict__ parts, int world, int64_t chunk,
                                                        bf16_t* __restrict__ out) {
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8; i < chunk; i += (int64_t)gridDim.x * 256 * 8) {
    float acc[8];
    const bool vec = i + 8 <= chunk;
    for (int r = 0; r < world; ++r) {
      const bf16_t* p = parts + (int64_t)r * chunk + i;
      float v[8];
      if (vec) {
        const uint4 q = *(const uint4*)p;
        const uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[2 * e] = __uint_as_float(u[e] << 16);
          v[2 * e + 1] = __uint_as_float(u[e] & 0xFFFF0000u);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = i + e < chunk ? bf2f(p[e]) : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = r == 0 ? v[e] : acc[e] + v[e];
    }
    if (vec) {
      *(uint4*)(out + i) = make_uint4(f2bf2(acc[0], acc[1]), f2bf2(acc[2], acc[3]), f2bf2(acc[4], acc[5]),
                                      f2bf2(acc[6], acc[7]));
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (i + e < chunk) out[i + e] = f2bf(acc[e]);
    }
  }
}

__global__ __launch_bounds__(256) void k_exchange_unpack(const bf16_t* __restrict__ in, int64_t n, float* __restrict__ x) {
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8; i < n; i += (int64_t)gridDim.x * 256 * 8) {
    if (i + 8 <= n && (((uintptr_t)(x + i)) & 15) == 0) {
      const uint4 q = *(const uint4*)(in + i);
      const uint32_t u[4] = {q.x, q.y, q.z, q.w};
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] = __uint_as_float(u[e] << 16);
        v[2 * e + 1] = __uint_as_float(u[e] & 0xFFFF0000u);
      }
      *(float4*)(x + i) = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)(x + i + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (i + e < n) x[i + e] = bf2f(in[i + e]);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Certified-band recompute of the sampling decode (MaskBand; SURVEY.md 7 "Hard parts" (ii)): one
// wave per listed (row, gene): logit = sum_k A[row][k] W[gene][k] in fp64 (each lane a strided
// slice of k in order, then a fixed-order wave reduction: deterministic) + bias[gene]; the mask bit
// becomes (float)logit > T, the correctly rounded fp32 logit against the reference's threshold.
// Packed bits are set / cleared with 32-bit atomics (several waves may share a word), u8 masks by
// byte stores. flips counts the bits the recompute changed.
// ---------------------------------------------------------------------------------------------
// one band element per 16-lane group (four per wave): fp64 dot of the fp32 rows in a fixed order
// (each lane a strided slice of float4s, then a fixed 16-lane tree) + bias; the group's first lane
// sets or clears the bit. H % 4 == 0 and 16-B aligned rows (decode_split3's preconditions).
__device__ __forceinline__ void band_fix_one(const uint2 rg, bool valid, int lane, const float* __restrict__ A,
                                             int64_t lda, const float* __restrict__ W, int64_t ldw,
                                             const float* __restrict__ bias, int H, uint8_t* bits, int64_t ldb,
                                             uint8_t* mask, int64_t ldm, unsigned* flips) {
  const int q = lane & 15;
  double acc = 0.0;
  if (valid) {
    const float4* a = (const float4*)(A + (int64_t)rg.x * lda);
    const float4* w = (const float4*)(W + (int64_t)rg.y * ldw);
    for (int k = q; k < H / 4; k += 16) {
      const float4 x = a[k], y = w[k];
      acc = fma((double)x.x, (double)y.x, acc);
      acc = fma((double)x.y, (double)y.y, acc);
      acc = fma((double)x.z, (double)y.z, acc);
      acc = fma((double)x.w, (double)y.w, acc);
    }
  }
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (!valid || q != 0) return;
  acc += (double)bias[rg.y];
  const bool pred = (float)acc > kMaskLogitThreshold;
  bool was;
  if (bits) {
    unsigned* word = (unsigned*)(bits + (int64_t)rg.x * ldb) + (rg.y >> 5);
    const unsigned bit = 1u << (rg.y & 31);
    const unsigned old = pred ? atomicOr(word, bit) : atomicAnd(word, ~bit);
    was = (old & bit) != 0;
  } else {
    uint8_t* p = mask + (int64_t)rg.x * ldm + rg.y;
    was = *p != 0;
    *p = pred ? 1 : 0;
  }
  if (was != pred) atomicAdd(flips, 1u);
}

// workgroups [0, kBandFixShardWgs): the shards (wave w takes shard w % kBandShards, its entries
// 4 (w / kBandShards) + group, + 4 waves / kBandShards, ...); the rest: one wave per tile's slots,
// four entries at a time, four consecutive tiles (row-major: one genome-row block) per workgroup.
// xcd: consecutive workgroups of ONE XCD take consecutive tile quads (the dispatcher deals
// workgroups round-robin over the 8 XCDs), so the activation rows of a row block's band entries --
// each row recurs in the lists of ~1/4 of its row's 215 tiles -- are fetched into one L2, not eight
constexpr int kBandFixShardWgs = 256;
__global__ __launch_bounds__(256) void k_band_fix(MaskBand band, int ntiles, const float* __restrict__ A, int64_t lda,
                                                const float* __restrict__ W, int64_t ldw, const float* __restrict__ bias,
                                                int H, uint8_t* bits, int64_t ldb, uint8_t* mask, int64_t ldm,
                                                unsigned* flips, int xcd) {
  const int lane = threadIdx.x & 63, grp = lane >> 4;
  if (blockIdx.x < kBandFixShardWgs) {
    const unsigned wave = blockIdx.x * 4 + (threadIdx.x >> 6), waves = kBandFixShardWgs * 4;
    const int sh = wave % kBandShards;
    const unsigned per = waves / kBandShards;
    const unsigned n = min(band.counts[sh], band.cap);
    const uint2* sl = band.list + (size_t)sh * band.cap;
    for (unsigned e0 = 4 * (wave / kBandShards); e0 < n; e0 += 4 * per) {
      const unsigned e = e0 + grp;
      band_fix_one(e < n ? sl[e] : make_uint2(0u, 0u), e < n, lane, A, lda, W, ldw, bias, H, bits, ldb, mask, ldm,
                   flips);
    }
    return;
  }
  const int nb = (int)gridDim.x - kBandFixShardWgs, b = (int)blockIdx.x - kBandFixShardWgs;
  int lb = b;
  if (xcd) {  // (kBandFixShardWgs % 8 == 0: b's XCD is blockIdx's)
    const int q = nb >> 3, r = nb & 7, x = b & 7;
    lb = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
  }
  const int t = lb * 4 + (threadIdx.x >> 6);
  if (t >= ntiles) return;
  const unsigned n = min(band.tcount[t], (unsigned)band.tslots);
  const uint2* tl = band.tlist + (size_t)t * band.tslots;
  for (unsigned e0 = 0; e0 < n; e0 += 4) {
    const unsigned e = e0 + grp;
    band_fix_one(e < n ? tl[e] : make_uint2(0u, 0u), e < n, lane, A, lda, W, ldw, bias, H, bits, ldb, mask, ldm,
                 flips);
  }
}

// Whole-block recompute of the blocks whose band entries overflowed the shard list (MaskBand.olist):
// a work item is 16 rows (fewer for H > 1024: the rows' fp32 activations fill at most 64 KB of LDS) x
// the block's 256 genes, one gene per thread; each logit sum_k A[row][k] W[gene][k] in fp64 in k
// order + bias[gene], the bit (float)logit > T as in k_band_fix. Packed bits leave as whole 32-bit
// words (one wave ballot per row: 64 genes = 2 words), so no atomics: the block's words belong to
// this item alone, and k_band_fix is done with them (stream order). Rows >= n are not written;
// genes >= G are 0 (the packed rows' pad bits), words past the row pitch are not written.
constexpr int kTileFixRows = 16;
__global__ __launch_bounds__(256) void k_band_tile_fix(const unsigned* __restrict__ olist,
                                                     const unsigned* __restrict__ ocount, int obn, unsigned oblocks,
                                                     const float* __restrict__ A, int64_t lda,
                                                     const float* __restrict__ W, int64_t ldw,
                                                     const float* __restrict__ bias, int H, int rows_per, int n, int G,
                                                     uint8_t* bits, int64_t ldb, uint8_t* mask, int64_t ldm,
                                                     unsigned* flips) {
  extern __shared__ __attribute__((aligned(16))) float sa[];  // [rows_per][H]
  const int subs = 256 / rows_per, lane = threadIdx.x & 63;
  const unsigned nblk = min(*ocount, oblocks), items = nblk * (unsigned)subs;
  GM2_DBG(*ocount <= oblocks, kDbgBandBlock);
  unsigned nflip = 0;
  for (unsigned it = blockIdx.x; it < items; it += gridDim.x) {
    const unsigned blk = olist[it / subs];
    GM2_DBG(blk < oblocks, kDbgBandBlock);
    const int m0 = (int)(blk / (unsigned)obn) * 256 + (int)(it % subs) * rows_per;
    const int g = (int)(blk % (unsigned)obn) * 256 + (int)threadIdx.x;
    __syncthreads();  // (the previous item's rows are read)
    for (int i = threadIdx.x; i < rows_per * H; i += 256) {
      const int r = i / H;
      sa[i] = m0 + r < n ? A[(int64_t)(m0 + r) * lda + (i - r * H)] : 0.f;
    }
    __syncthreads();
    double acc[kTileFixRows];
#pragma unroll
    for (int r = 0; r < kTileFixRows; ++r) acc[r] = 0.0;
    if (g < G) {
      const float4* w = (const float4*)(W + (int64_t)g * ldw);
      for (int k4 = 0; k4 < H / 4; ++k4) {
        const float4 y = w[k4];
#pragma unroll
        for (int r = 0; r < kTileFixRows; ++r) {
          if (r < rows_per) {
            const float4 x = *(const float4*)(sa + r * H + 4 * k4);
            acc[r] = fma((double)x.x, (double)y.x, acc[r]);
            acc[r] = fma((double)x.y, (double)y.y, acc[r]);
            acc[r] = fma((double)x.z, (double)y.z, acc[r]);
            acc[r] = fma((double)x.w, (double)y.w, acc[r]);
          }
        }
      }
    }
    const double b = g < G ? (double)bias[g] : 0.0;
#pragma unroll
    for (int r = 0; r < kTileFixRows; ++r) {
      const int row = m0 + r;
      if (r >= rows_per || row >= n) continue;  // (uniform)
      const bool pred = g < G && (float)(acc[r] + b) > kMaskLogitThreshold;
      if (bits) {
        const uint64_t bal = __ballot(pred);
        const int64_t byte = (int64_t)(g - lane) / 8 + 4 * (lane & 1);  // word (lane & 1) of the wave's 64 genes
        if (lane < 2 && byte + 4 <= ldb) {
          unsigned* word = (unsigned*)(bits + (int64_t)row * ldb + byte);
          const unsigned v = (unsigned)(bal >> (32 * lane));
          nflip += __popc(*word ^ v);
          *word = v;
        }
      } else if (g < G) {
        uint8_t* p = mask + (int64_t)row * ldm + g;
        nflip += (*p != 0) != pred;
        *p = pred ? 1 : 0;
      }
    }
  }
  if (nflip) atomicAdd(flips, nflip);
}

// the decode call's counters -> the workspace's cumulative ones: cum[0] split tiles, [1] exact
// tiles, [2] band elements found, [3] bits the recompute flipped, [4] band elements beyond the
// list's capacity (left as the kernels decided them), [5] decodes with split or single tiles, [6]
// without, [7] single-product tiles
__global__ __launch_bounds__(64) void k_decode_stats(const unsigned* __restrict__ tiles_split,
                                                     const unsigned* __restrict__ tiles_exact,
                                                     const unsigned* __restrict__ tiles_single,
                                                     const unsigned* __restrict__ counts,
                                                     const unsigned* __restrict__ tfound,
                                                     const unsigned* __restrict__ flips, unsigned cap,
                                                     unsigned long long* cum, const unsigned* __restrict__ ocount,
                                                     unsigned long long* ocum) {
  const int t = threadIdx.x;
  unsigned long long a = t < kSplitShards ? tiles_split[t] : 0ull, b = t < kSplitShards ? tiles_exact[t] : 0ull;
  unsigned long long g = t < kSplitShards ? tiles_single[t] : 0ull;
  const unsigned c = t < kBandShards ? counts[t] : 0u;
  unsigned long long found = (unsigned long long)c + (t < kBandShards ? tfound[t] : 0u), over = c > cap ? c - cap : 0u;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
    g += __shfl_xor(g, o, 64);
    found += __shfl_xor(found, o, 64);
    over += __shfl_xor(over, o, 64);
  }
  if (t == 0) {
    cum[0] += a;
    cum[1] += b;
    cum[2] += found;
    cum[3] += *flips;
    cum[4] += over;
    cum[a || g ? 5 : 6] += 1;
    cum[7] += g;
    *ocum += *ocount;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_transpose(const T* __restrict__ src, int64_t lds_, T* __restrict__ dst,
                                                 int64_t ldd) {
  constexpr int EPC = 16 / sizeof(T), CPR = 64 / EPC, RPP = 256 / CPR;
  __shared__ __attribute__((aligned(16))) T tile[64][64 + EPC];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int ch = threadIdx.x % CPR, rr = threadIdx.x / CPR;
#pragma unroll
  for (int p = 0; p < 64; p += RPP)
    *(uint4*)&tile[p + rr][ch * EPC] = *(const uint4*)(src + (r0 + p + rr) * lds_ + c0 + ch * EPC);
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 64; p += RPP) {
    const int c = p + rr;
    T v[EPC];
#pragma unroll
    for (int j = 0; j < EPC; ++j) v[j] = tile[ch * EPC + j][c];
    *(uint4*)(dst + (c0 + c) * ldd + r0 + ch * EPC) = *(const uint4*)v;
  }
}

// out[c] = sum_r part[r][c]: 64 columns x 4 row groups per block, fixed order (deterministic)
__global__ __launch_bounds__(256) void k_colsum2(const float* __restrict__ part, int rows, int64_t ld, int64_t n,
                                               float* __restrict__ out0, float* __restrict__ out1, int64_t nsplit) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + cl;
  float s = 0.f;
  if (c < n) {
    int r = rg;
    for (; r + 60 < rows; r += 64) {  // 16 rows' loads in flight, summed in row order
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = part[(int64_t)(r + 4 * u) * ld + c];
#pragma unroll
      for (int u = 0; u < 16; ++u) s += v[u];
    }
    for (; r < rows; r += 4) s += part[(int64_t)r * ld + c];
  }
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && c < n) {
    const float v = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
    if (c < nsplit) out0[c] = v;
    else out1[c - nsplit] = v;
  }
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
template <typename T>
void launch_gather_rows(const uint8_t* data, int64_t ld_data, const int32_t* rows, int B, int G, T* X, int64_t ldx,
                        int Gp, int Bp, uint32_t* xbits, int64_t ldxb, hipStream_t s) {
  // (the gather reads columns < roundup(G, 8) only: ld_data need not cover Gp's extra padding)
  if (Gp % 128 || Bp % 64 || ld_data % 16 || ld_data < G || ((uintptr_t)data & 15) || (xbits && ldxb * 32 < Gp))
    throw Gm2Error("gather: bad layout (Gp=%d Bp=%d ld=%lld)", Gp, Bp, (long long)ld_data);
  hipLaunchKernelGGL(k_gather<T>, dim3((Gp + 511) / 512, Bp / 32), dim3(256), 0, s, data, ld_data, rows, B, G, Gp, X,
                     ldx, xbits, ldxb);
  GM2_CHECK_LAUNCH();
}

__global__ __launch_bounds__(256) void k_resident_rows(const int32_t* __restrict__ rows, int n, int nfill, int zero_row,
                                                     int32_t* __restrict__ ridx) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < nfill) ridx[i] = i < n ? (rows ? rows[i] : i) : zero_row;
  if (rows && i < n) GM2_DBG(rows[i] >= 0 && rows[i] < zero_row, kDbgResidentRows);
}

void launch_resident_rows(const int32_t* rows, int n, int nfill, int64_t S, int32_t* ridx, hipStream_t s) {
  if (n > nfill || S < 0 || S > INT32_MAX) throw Gm2Error("resident rows: n=%d fill=%d S=%lld", n, nfill, (long long)S);
  hipLaunchKernelGGL(k_resident_rows, dim3((nfill + 255) / 256), dim3(256), 0, s, rows, n, nfill, (int)S, ridx);
  GM2_CHECK_LAUNCH();
}

void launch_bn_fwd_partial(const float* slabs, int S, int64_t slab, int64_t ld, const float* bias, int B, int H,
                           float* Y, float* part, hipStream_t s) {
  if (H % 64) throw Gm2Error("bn: H %% 64");
  const int nch = (B + kBnRowChunk - 1) / kBnRowChunk;
  hipLaunchKernelGGL(k_bn_fwd_partial, dim3(H / 64, nch), dim3(256), 0, s, slabs, S, slab, ld, bias, B, H, Y,
                     (float2*)part);
  GM2_CHECK_LAUNCH();
}

void launch_bn_bwd_partial(const float* dslabs, int S, int64_t slab, const float* Y, int64_t ld, const float* save,
                           const float* gamma, const float* beta, int B, int H, float* part, float* dsum,
                           hipStream_t s) {
  if (H % 64) throw Gm2Error("bn: H %% 64");
  const int nch = (B + kBnRowChunk - 1) / kBnRowChunk;
  hipLaunchKernelGGL(k_bn_bwd_partial, dim3(H / 64, nch), dim3(256), 0, s, dslabs, S, slab, Y, ld, save, gamma,
                     beta, B, H, (float2*)part, dsum);
  GM2_CHECK_LAUNCH();
}

template <typename T>
void launch_reparam(const float* slabs, int S, int64_t slab, int L, const float* bmu, const float* blv,
                    const float* eps, int B, int Bp, float* HD, T* Z, int64_t ldz, T* ZT, int64_t ldzt, int Lrows,
                    float* kl_part, hipStream_t s) {
  (void)Lrows;
  if (L > 256 || Bp % kReparamRows) throw Gm2Error("reparam: latent_dim <= 256");
  hipLaunchKernelGGL(k_reparam<T>, dim3(Bp / kReparamRows), dim3(256), 0, s, slabs, S, slab, L, bmu, blv, eps, B, HD, Z, ldz,
                     ZT, ldzt, kl_part);
  GM2_CHECK_LAUNCH();
}

template <typename T>
void launch_reparam_bwd(const float* dzslabs, int S, int64_t slab, int64_t ldslab, const float* HD, const float* eps,
                        const float* scal, int B, int Bp, int L, T* dH, int64_t ldh, const float* dmu_ext,
                        const float* dlv_ext, float* colpart, hipStream_t s) {
  if (L > 256 || 256 % L) throw Gm2Error("reparam_bwd: latent_dim must divide 256");
  hipLaunchKernelGGL(k_reparam_bwd<T>, dim3(Bp / kReparamRows), dim3(256), 0, s, dzslabs, S, slab, ldslab, HD, eps, scal, B, L,
                     dH, ldh, dmu_ext, dlv_ext, colpart);
  GM2_CHECK_LAUNCH();
}

void launch_reparameterize(int64_t n, const float* mu, const float* lv, const float* eps, float* z, const float* dz,
                           float* dmu, float* dlv, hipStream_t s) {
  if (n <= 0) return;
  const int64_t nb = std::min<int64_t>(4096, (n + 255) / 256);
  hipLaunchKernelGGL(k_reparameterize, dim3((unsigned)nb), dim3(256), 0, s, n, mu, lv, eps, z, dz, dmu, dlv);
  GM2_CHECK_LAUNCH();
}

template <typename T>
void launch_sigmoid_bwd(const float* p, const float* dp, int64_t ldp, int B, int Bp, int G, int Gp, T* dL, int64_t ldd,
                        float* colpart, hipStream_t s) {
  hipLaunchKernelGGL(k_sigmoid_bwd<T>, dim3((Gp + 255) / 256, Bp / 64), dim3(256), 0, s, p, dp, ldp, B, G, Gp, dL, ldd,
                     colpart);
  GM2_CHECK_LAUNCH();
}

void launch_colsum(const float* part, int rows, int64_t ld, int64_t n, float* out0, float* out1, int64_t nsplit,
                   hipStream_t s) {
  if ((n + 63) / 64 > INT32_MAX) throw Gm2Error("colsum: %lld columns", (long long)n);
  hipLaunchKernelGGL(k_colsum2, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, s, part, rows, ld, n, out0, out1 ? out1 : out0,
                     out1 ? nsplit : n);
  GM2_CHECK_LAUNCH();
}

template <typename T>
void launch_bn_fwd_apply(const float* Y, int64_t ld, const float* part, int B, int Bp, int H, int train,
                         const float* gamma, const float* beta, float* rmean, float* rvar, float* save, T* A,
                         hipStream_t s, const double* sync) {
  if (H % 128 || ld % 4 || Bp % 64 || B <= 0) throw Gm2Error("bn_fwd_apply: H %% 128, ld %% 4, Bp %% 64, B > 0");
  hipLaunchKernelGGL(k_bn_fwd_apply<T>, dim3((H + 255) / 256, Bp / 64), dim3(256), 0, s, Y, ld, (const float2*)part,
                     B, H, train, gamma, beta, rmean, rvar, save, A, sync);
  GM2_CHECK_LAUNCH();
}

void launch_bn_sync_pack(const float* part, int B, int H, int mode, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_bn_sync_pack, dim3((H + 255) / 256), dim3(256), 0, s, (const float2*)part, B, H, mode, out);
  GM2_CHECK_LAUNCH();
}

void launch_bn_sync_running(const double* sync, int H, float* rmean, float* rvar, hipStream_t s) {
  hipLaunchKernelGGL(k_bn_sync_running, dim3((H + 255) / 256), dim3(256), 0, s, sync, H, rmean, rvar);
  GM2_CHECK_LAUNCH();
}
template <typename T>
void launch_bn_bwd_apply(const float* da, const float* Y, int64_t ld, const float* part, int B, int Bp, int H,
                         int train, const float* save, const float* gamma, const float* beta, float* dgamma,
                         float* dbeta, T* dY, float* colpart, hipStream_t s, const double* sync, T* dYT,
                         int64_t ldt) {
  if (H % 128 || ld % 4 || Bp % 64 || B <= 0) throw Gm2Error("bn_bwd_apply: H %% 128, ld %% 4, Bp %% 64, B > 0");
  if (dYT && (sizeof(T) != 2 || ldt % 8 || ldt < Bp)) throw Gm2Error("bn_bwd_apply: transposed output (bf16, ldt)");
  hipLaunchKernelGGL(k_bn_bwd_apply<T>, dim3((H + 255) / 256, Bp / 64), dim3(256), 0, s, da, Y, ld,
                     (const float2*)part, B, H, train, save, gamma, beta, dgamma, dbeta, dY, colpart, sync, dYT, ldt);
  GM2_CHECK_LAUNCH();
}

void launch_split3(const float* X, int64_t ldx, int rows, int rows_pad, int K, bf16_t* out, int64_t ldo, float* rn,
                   unsigned* blk, hipStream_t s, bf16_t* out1) {
  if (K % 32 || ldx % 4 || ldo % 8 || ldo < 2 * K || rows > rows_pad || rows_pad % 256 || (((uintptr_t)X) & 15) ||
      (((uintptr_t)out) & 15) || (((uintptr_t)out1) & 15))
    throw Gm2Error("split3: K %d, ld %lld / %lld, rows %d / %d", K, (long long)ldx, (long long)ldo, rows, rows_pad);
  hipLaunchKernelGGL(k_split3, dim3(rows_pad / 16), dim3(256), 0, s, X, ldx, rows, K, out, ldo, rn, blk, out1);
  GM2_CHECK_LAUNCH();
}

static unsigned elementwise_grid(int64_t n) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 2047) / 2048, 8192));
}

void launch_exchange_pack(const float* x, int64_t n, bf16_t* out, int64_t n_pad, hipStream_t s) {
  if (n < 0 || n_pad < n || (((uintptr_t)out) & 15)) throw Gm2Error("exchange pack: n %lld, n_pad %lld", (long long)n, (long long)n_pad);
  if (n_pad == 0) return;
  hipLaunchKernelGGL(k_exchange_pack, dim3(elementwise_grid(n_pad)), dim3(256), 0, s, x, n, out, n_pad);
  GM2_CHECK_LAUNCH();
}

void launch_exchange_ranksum(const bf16_t* parts, int world, int64_t chunk, bf16_t* out, hipStream_t s) {
  if (world < 1 || chunk < 0 || chunk % 8 || (((uintptr_t)parts | (uintptr_t)out) & 15))
    throw Gm2Error("exchange ranksum: world %d, chunk %lld (a multiple of 8, 16-B aligned buffers)", world,
                   (long long)chunk);
  if (chunk == 0) return;
  hipLaunchKernelGGL(k_exchange_ranksum, dim3(elementwise_grid(chunk)), dim3(256), 0, s, parts, world, chunk, out);
  GM2_CHECK_LAUNCH();
}

void launch_exchange_unpack(const bf16_t* in, int64_t n, float* x, hipStream_t s) {
  if (n < 0 || (((uintptr_t)in) & 15)) throw Gm2Error("exchange unpack: n %lld", (long long)n);
  if (n == 0) return;
  hipLaunchKernelGGL(k_exchange_unpack, dim3(elementwise_grid(n)), dim3(256), 0, s, in, n, x);
  GM2_CHECK_LAUNCH();
}

void launch_band_fix(const MaskBand& band, int ntiles, const float* A, int64_t lda, const float* W, int64_t ldw,
                     const float* bias, int H, uint8_t* bits, int64_t ldb, uint8_t* mask, int64_t ldm, unsigned* flips,
                     hipStream_t s) {
  if ((!bits && !mask) || (bits && (ldb & 3)))
    throw Gm2Error("band fix: an output (packed bits with 4-B aligned rows, or a u8 mask) is required");
  if (!band.counts || !band.list || !band.cap || ntiles < 0 || (ntiles && (!band.tlist || !band.tcount || band.tslots <= 0)))
    throw Gm2Error("band fix: shard list and counters (and tile slots for %d tiles) required", ntiles);
  // (a fixed grid for the shards, the counts live on the device: 16 waves per shard; then one wave per tile)
  static_assert((kBandFixShardWgs * 4) % kBandShards == 0, "band fix grid");
  static_assert(kBandFixShardWgs % 8 == 0, "band fix: XCD-aware tile order");
  const unsigned grid = kBandFixShardWgs + (unsigned)((ntiles + 3) / 4);
  // env GM2_BANDFIX_LINEAR=1: tile quads in dispatch order (A/B of the XCD-aware order)
  static const int xcd = std::getenv("GM2_BANDFIX_LINEAR") ? 0 : 1;
  hipLaunchKernelGGL(k_band_fix, dim3(grid), dim3(256), 0, s, band, ntiles, A, lda, W, ldw, bias, H, bits, ldb, mask,
                     ldm, flips, xcd);
  GM2_CHECK_LAUNCH();
}

// packed mask bits (bit g % 8 of byte g / 8, rows of ldb bytes) -> u8 rows of ldm bytes at any
// alignment (gm2_decode_mask): a workgroup per row at a time -- the row's packed bytes staged in LDS
// by 16-B loads, then one thread per 4-B aligned output dword (the first and last dwords of a row,
// shared with its neighbours, by bytes), so every wave instruction writes 256 contiguous bytes
__global__ __launch_bounds__(256) void k_expand_bits(const uint8_t* __restrict__ bits, int64_t ldb, int n, int G,
                                                   uint8_t* __restrict__ out, int64_t ldm) {
  extern __shared__ __attribute__((aligned(16))) char lrow[];
  const int nb = (G + 7) / 8, nv = (nb + 15) / 16;  // packed bytes of a row, 16-B pieces
  for (int r = blockIdx.x; r < n; r += gridDim.x) {
    const uint8_t* br = bits + (int64_t)r * ldb;
    __syncthreads();  // (the previous row's reads of lrow are done)
    for (int v = threadIdx.x; v < nv; v += 256) *(uint4*)(lrow + 16 * v) = *(const uint4*)(br + 16 * v);
    __syncthreads();
    uint8_t* row = out + (int64_t)r * ldm;
    const int a = (int)((uintptr_t)row & 3);
    const int nd = (G + a + 3) / 4;
    for (int k = threadIdx.x; k < nd; k += 256) {
      const int c0 = 4 * k - a;  // the dword's first column (-a at k = 0: those bytes are the row before's)
      uint32_t x = 0;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int c = c0 + t;
        if (c >= 0 && c < G) x |= ((uint32_t)((uint8_t)lrow[c >> 3] >> (c & 7)) & 1u) << t;
      }
      if (c0 >= 0 && c0 + 3 < G) {
        *(uint32_t*)(row + c0) = (x * 0x00204081u) & 0x01010101u;  // (row - a + 4k: aligned)
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (c0 + t >= 0 && c0 + t < G) row[c0 + t] = (uint8_t)((x >> t) & 1u);
      }
    }
  }
}

void launch_expand_bits(const uint8_t* bits, int64_t ldb, int n, int G, uint8_t* out, int64_t ldm, hipStream_t s) {
  if (!bits || !out || n < 0 || G < 0 || ldb * 8 < G || ldm < G) throw Gm2Error("expand bits: bad rows");
  const int64_t lds = round_up((G + 7) / 8, 16);
  if (ldb < lds || (ldb & 15) || (((uintptr_t)bits) & 15)) throw Gm2Error("expand bits: rows must be 16-B pieces");
  if (lds > 64 * 1024) throw Gm2Error("expand bits: %lld genes per row", (long long)G);
  if (n == 0 || G == 0) return;
  hipLaunchKernelGGL(k_expand_bits, dim3((unsigned)std::min(n, 4096)), dim3(256), (unsigned)lds, s, bits, ldb, n, G,
                     out, ldm);
  GM2_CHECK_LAUNCH();
}

void launch_decode_stats(const unsigned* tiles_split, const unsigned* tiles_exact, const unsigned* tiles_single,
                         const unsigned* counts, const unsigned* tfound, const unsigned* flips, unsigned cap,
                         unsigned long long* cum, const unsigned* ocount, unsigned long long* ocum, hipStream_t s) {
  static_assert(kSplitShards <= 64 && kBandShards <= 64, "one wave");
  hipLaunchKernelGGL(k_decode_stats, dim3(1), dim3(64), 0, s, tiles_split, tiles_exact, tiles_single, counts, tfound, flips, cap,
                     cum, ocount, ocum);
  GM2_CHECK_LAUNCH();
}

void launch_band_tile_fix(const MaskBand& band, const float* A, int64_t lda, const float* W, int64_t ldw,
                          const float* bias, int H, int n, int G, uint8_t* bits, int64_t ldb, uint8_t* mask,
                          int64_t ldm, unsigned* flips, hipStream_t s) {
  if ((!bits && !mask) || (bits && (ldb & 3)) || H < 4 || H % 4 || (((uintptr_t)W | (uintptr_t)(ldw * 4)) & 15))
    throw Gm2Error("band tile fix: packed bits with 4-B aligned rows or a u8 mask, H %% 4 == 0, 16-B aligned weight rows");
  if (!band.olist || !band.ocount || band.obn <= 0 || !band.oblocks || n < 0 || G < 0)
    throw Gm2Error("band tile fix: the overflow block list and counter required");
  // rows per work item: a power of two <= 16 whose fp32 rows fit 64 KB of LDS
  int rows_per = kTileFixRows;
  while (rows_per > 1 && (int64_t)rows_per * H * 4 > 65536) rows_per /= 2;
  const size_t lds = (size_t)rows_per * H * 4;
  if (lds > 65536) throw Gm2Error("band tile fix: hidden width %d too large", H);
  // (<= 64 KB: within the default dynamic-LDS limit, no attribute needed)
  hipLaunchKernelGGL(k_band_tile_fix, dim3(512), dim3(256), lds, s, band.olist, band.ocount, band.obn, band.oblocks, A,
                     lda, W, ldw,
                     bias, H, rows_per, n, G, bits, ldb, mask, ldm, flips);
  GM2_CHECK_LAUNCH();
}

template <typename T>
void launch_transpose(const T* src, int64_t lds_, int R, int Cn, T* dst, int64_t ldd, hipStream_t s) {
  if (R % 64 || Cn % 64 || (lds_ * sizeof(T)) % 16 || (ldd * sizeof(T)) % 16)
    throw Gm2Error("transpose: %d x %d block, pitches must be 16-B multiples", R, Cn);
  hipLaunchKernelGGL(k_transpose<T>, dim3(Cn / 64, R / 64), dim3(256), 0, s, src, lds_, dst, ldd);
  GM2_CHECK_LAUNCH();
}

void launch_fwd_tail(const float* lpart, int nl, const float* kpart, int nk, double* loss, const float* cpart, int rows,
                     int64_t ld, int64_t n, float* cout, int* hdr, int hv0, int hv1, hipStream_t s) {
  const int64_t cb = cout ? (n + 63) / 64 : 0;
  hipLaunchKernelGGL(k_fwd_tail, dim3((unsigned)(1 + cb)), dim3(256), 0, s, lpart, nl, kpart, nk, loss, cpart, rows, ld,
                     n, cout, hdr, hv0, hv1);
  GM2_CHECK_LAUNCH();
}


template <typename T>
void launch_shadow_sync(const TensorTable& tt, const float* params, hipStream_t s) {
  if (tt.n <= 0) return;
  const TensorDesc& last = tt.t[tt.n - 1];
  const int64_t tiles = last.tile0 + ((last.rows + 63) / 64) * ((last.cols + 63) / 64);
  hipLaunchKernelGGL(k_shadow_sync<T>, dim3((unsigned)tiles), dim3(256), 0, s, tt, params);
  GM2_CHECK_LAUNCH();
}

template <typename T>
void launch_adam_fused(const TensorTable& tt, const float* grads, float* params, float* m, float* v, const float* scal,
                       const float* clip, hipStream_t s, int max_grid, float* scal_copy) {
  const TensorDesc& last = tt.t[tt.n - 1];
  const int64_t blocks = last.tile0 + (last.rows * last.cols + 4095) / 4096;
  for (int i = 0; i < tt.n; ++i)
    if (tt.t[i].off % 4) throw Gm2Error("adam: tensor offset not 16-B aligned");
  const int64_t grid = max_grid > 0 ? std::min<int64_t>(blocks, max_grid) : blocks;
  TimedLaunch tl(kKcAdam, s);
  hipLaunchKernelGGL(k_adam_fused<T>, dim3((unsigned)grid), dim3(256), 0, s, tt, grads, params, m, v, scal, clip,
                     blocks, scal_copy);
  GM2_CHECK_LAUNCH();
}

void launch_slab_sum(const float* slabs, int S, int64_t slab, int M, int N, float* C0, float* C1, int msplit,
                     int64_t ldc, hipStream_t s) {
  if (slab % 4) throw Gm2Error("slab_sum: slab %% 4");
  const int64_t nb = std::min<int64_t>(4096, ((int64_t)M * N / 4 + 255) / 256);
  hipLaunchKernelGGL(k_slab_sum, dim3((unsigned)nb), dim3(256), 0, s, slabs, S, slab, M, N, C0, C1 ? C1 : C0,
                     C1 ? msplit : (1 << 30), ldc);
  GM2_CHECK_LAUNCH();
}

int grad_stats_blocks(int64_t n) { return (int)std::min<int64_t>(2048, std::max<int64_t>(1, (n + 255) / 256)); }

void launch_grad_stats(const float* params, const float* grads, int64_t n, const float* scal, double* part,
                       int nblocks, const NormAhead& na, hipStream_t s) {
  if (na.hdr && !(0 <= na.lo0 && na.lo0 <= na.hi0 && na.hi0 <= na.lo9 && na.lo9 <= na.hi9 && na.hi9 <= n))
    throw Gm2Error("grad_stats: bad skip ranges");
  hipLaunchKernelGGL(k_grad_stats, dim3(nblocks), dim3(256), 0, s, params, grads, n, scal, part, na);
  GM2_CHECK_LAUNCH();
}

void launch_grad_finalize(const double* part, int nblocks, const float* scal, float* clip_out, double* l1abs,
                          const NormAhead& na, hipStream_t s) {
  hipLaunchKernelGGL(k_grad_finalize, dim3(1), dim3(256), 0, s, part, nblocks, scal, clip_out, l1abs, na);
  GM2_CHECK_LAUNCH();
}

#define GM2_INST(T)                                                                                             \
  template void launch_gather_rows<T>(const uint8_t*, int64_t, const int32_t*, int, int, T*, int64_t, int, int,  \
                                      uint32_t*, int64_t, hipStream_t);                                         \
  template void launch_reparam<T>(const float*, int, int64_t, int, const float*, const float*, const float*,   \
                                  int, int, float*, T*, int64_t, T*, int64_t, int, float*, hipStream_t);        \
  template void launch_reparam_bwd<T>(const float*, int, int64_t, int64_t, const float*, const float*,         \
                                      const float*, int, int, int, T*, int64_t, const float*, const float*,     \
                                      float*, hipStream_t);                                                     \
  template void launch_sigmoid_bwd<T>(const float*, const float*, int64_t, int, int, int, int, T*, int64_t,     \
                                      float*, hipStream_t);                                                     \
  template void launch_shadow_sync<T>(const TensorTable&, const float*, hipStream_t);                          \
  template void launch_bn_fwd_apply<T>(const float*, int64_t, const float*, int, int, int, int, const float*,   \
                                       const float*, float*, float*, float*, T*, hipStream_t, const double*);    \
  template void launch_bn_bwd_apply<T>(const float*, const float*, int64_t, const float*, int, int, int, int,    \
                                       const float*, const float*, const float*, float*, float*, T*, float*,    \
                                       hipStream_t, const double*, T*, int64_t);                                \
  template void launch_transpose<T>(const T*, int64_t, int, int, T*, int64_t, hipStream_t);                    \
  template void launch_adam_fused<T>(const TensorTable&, const float*, float*, float*, float*, const float*,    \
                                     const float*, hipStream_t, int, float*);
GM2_INST(float)
GM2_INST(bf16_t)
#undef GM2_INST

#ifdef GM2_DEBUG
GM2_DBG_TAKE_FN(dbg_take_kernels)
#endif

}  // namespace gm2
