// BatchNorm1d finalisation (training/model.py:66-86, nn.BatchNorm1d train mode), shared by the
// apply kernels (kernels.hip) and by the producers whose LAST-ARRIVING workgroup finalises a block of
// columns (the hidden-layer GEMM epilogues in gemm.hip, the split-K statistics passes in kernels.hip).
//
// Statistics arrive as per-128-row-chunk partials part[chunk][H] (float2):
//   forward : (chunk mean, chunk M2) of the pre-BN output y
//   backward: (sum do, sum (y - mean) do), do = dA * [bn output > 0]
// The last-arriver hand-off (BnFin): every producing workgroup stores its partials write-through
// (sc1), drains them (s_waitcnt vmcnt(0)), joins a workgroup barrier, and one lane adds 1 to the
// column block's arrival counter (agent scope). The workgroup whose add returns arrivals - 1 reads
// every chunk's partials of its columns with sc1 loads, merges them in chunk order in fp64 (the same
// arithmetic as the apply kernels' own merge: bit-identical coefficients), writes the per-column
// coefficient table and the side outputs (batch mean / invstd, running statistics; dgamma / dbeta),
// and resets the counter to 0 for the next launch. No workgroup waits on another (placement- and
// residency-independent); the hand-off is MI355X_MICROARCH.md § visibility, valid-forms row 1.
#pragma once
#include "gm2_common.hpp"

namespace gm2 {

constexpr double kBnEps = 1e-5;       // nn.BatchNorm1d default eps
constexpr double kBnMomentum = 0.1;   // nn.BatchNorm1d default momentum
constexpr int kBnChunk = 128;         // rows per partial-statistics chunk (= kBnRowChunk)

typedef __attribute__((address_space(1))) unsigned long long gu64_t;
typedef __attribute__((address_space(1))) int gi32_t;

// Chan's parallel merge of per-chunk (mean, M2) -> batch mean and biased variance, in two passes
// (mean = sum n_c mean_c / B ; M2 = sum M2_c + n_c (mean_c - mean)^2), fp64. ld(ch) returns chunk
// ch's float2. Up to 32 chunks (B <= 4096) the partials are loaded once, all in flight.
template <class LD>
__device__ __forceinline__ void bn_merge_ld(LD ld, int B, double& mean, double& var) {
  const int nch = (B + kBnChunk - 1) / kBnChunk;
  double s = 0.0, mu, M2 = 0.0;
  if (nch <= 32) {
    // branch-free: chunks past nch re-read the last chunk with weight 0 (exact no-ops)
    float2 p[32];
#pragma unroll
    for (int ch = 0; ch < 32; ++ch) p[ch] = ld(min(ch, nch - 1));
#pragma unroll
    for (int ch = 0; ch < 32; ++ch) {
      const double nb = (double)max(0, min(kBnChunk, B - ch * kBnChunk));
      s += nb * (double)p[ch].x;
    }
    mu = s / (double)B;
#pragma unroll
    for (int ch = 0; ch < 32; ++ch) {
      const double nb = (double)max(0, min(kBnChunk, B - ch * kBnChunk));
      const double dlt = (double)p[ch].x - mu;
      M2 += (ch < nch ? (double)p[ch].y : 0.0) + nb * dlt * dlt;
    }
    mean = mu;
    var = M2 / (double)B;
    return;
  }
#pragma unroll 8
  for (int ch = 0; ch < nch; ++ch) {
    const double nb = (double)min(kBnChunk, B - ch * kBnChunk);
    s += nb * (double)ld(ch).x;
  }
  mu = s / (double)B;
#pragma unroll 8
  for (int ch = 0; ch < nch; ++ch) {
    const double nb = (double)min(kBnChunk, B - ch * kBnChunk);
    const float2 p = ld(ch);
    const double dlt = (double)p.x - mu;
    M2 += (double)p.y + nb * dlt * dlt;
  }
  mean = mu;
  var = M2 / (double)B;
}

// backward sums (sum do, sum (y - mean) do) over the chunks, fp64, chunk order
template <class LD>
__device__ __forceinline__ void bn_bwd_sums_ld(LD ld, int B, double& s1, double& s2) {
  const int nch = (B + kBnChunk - 1) / kBnChunk;
  s1 = 0.0;
  s2 = 0.0;
  if (nch <= 32) {  // every chunk partial in flight at once, summed in chunk order
    float2 p[32];
#pragma unroll
    for (int ch = 0; ch < 32; ++ch) p[ch] = ld(min(ch, nch - 1));
#pragma unroll
    for (int ch = 0; ch < 32; ++ch) {
      s1 += ch < nch ? (double)p[ch].x : 0.0;
      s2 += ch < nch ? (double)p[ch].y : 0.0;
    }
    return;
  }
#pragma unroll 8
  for (int ch = 0; ch < nch; ++ch) {
    const float2 p = ld(ch);
    s1 += p.x;
    s2 += p.y;
  }
}

// train-mode forward: save <- (mean, invstd), running statistics updated (momentum 0.1, unbiased
// variance), returns (alpha, beta') with y * alpha + beta' = the BatchNorm output
__device__ __forceinline__ float2 bn_fwd_train_coef(double mean, double var, double n, int H, int col,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    float* rmean, float* rvar, float* save, bool own) {
  const float invstd = (float)(1.0 / sqrt(var + kBnEps));
  const float meanf = (float)mean;
  if (own) {
    save[col] = meanf;
    save[H + col] = invstd;
    const double unb = n > 1.0 ? var * n / (n - 1.0) : var;
    rmean[col] = (float)(kBnMomentum * mean + (1.0 - kBnMomentum) * (double)rmean[col]);
    rvar[col] = (float)(kBnMomentum * unb + (1.0 - kBnMomentum) * (double)rvar[col]);
  }
  const float alpha = invstd * gamma[col];
  return make_float2(alpha, fmaf(-meanf, alpha, beta[col]));
}

// backward coefficients of column col: [mean, alpha, beta', grad_mean, proj_scale] with
//   dx = (do - grad_mean - (y - mean) * proj_scale) * alpha ,  do = da * [y * alpha + beta' > 0]
// (g1, g2, nb: the sums and row count the batch coupling uses -- this batch's, or SyncBN's global)
__device__ __forceinline__ void bn_bwd_coef(double g1, double g2, double nb, int train, int H, int col,
                                            const float* __restrict__ save, const float* __restrict__ gamma,
                                            const float* __restrict__ beta, float (&cf)[5]) {
  const float mean = save[col], invstd = save[H + col];
  const float alpha = invstd * gamma[col];
  cf[0] = mean;
  cf[1] = alpha;
  cf[2] = fmaf(-mean, alpha, beta[col]);
  cf[3] = train ? (float)(g1 / nb) : 0.f;
  cf[4] = train ? (float)(g2 * (double)invstd * invstd / nb) : 0.f;
}

// ---- the last-arriver hand-off ----
struct BnFin {
  int mode = 0;                  // 0 off; 1 forward; 2 backward
  int train = 1;
  int B = 0, H = 0;              // batch rows, columns
  const float2* part = nullptr;  // [chunk][H]
  int* cnt = nullptr;            // arrival counter per column block (zero between launches)
  float* coef = nullptr;         // forward: float2 [H] (alpha, beta'); backward: float [5][H]
  const float* gamma = nullptr;
  const float* beta = nullptr;
  float* rmean = nullptr;        // forward
  float* rvar = nullptr;
  float* save = nullptr;         // forward: written; backward: read
  float* dgamma = nullptr;       // backward
  float* dbeta = nullptr;
};

__device__ __forceinline__ void st_sc1_f2(float2* p, float2 v) {
  __hip_atomic_store((gu64_t*)p, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float2 ld_sc1_f2(const float2* p) {
  return __builtin_bit_cast(float2, __hip_atomic_load((gu64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// Register-light forms of the two merges (one partial in registers at a time): the same
// arithmetic in the same order as bn_merge_ld / bn_bwd_sums_ld (their chunks past nch add exact
// zeros), for the last arriver of a GEMM epilogue, whose partials wait in LDS. (Inlined with 32
// partials in flight, the merge raised the 128x128 store kernel from 72 VGPRs to 128 with scratch
// spills, and it could no longer run beside the deferred output-layer update: profiles/r04_bn_fin_ab.txt.)
template <class LD>
__device__ __forceinline__ void bn_merge_seq(LD ld, int B, double& mean, double& var) {
  const int nch = (B + kBnChunk - 1) / kBnChunk;
  double s = 0.0, M2 = 0.0;
#pragma unroll 1
  for (int ch = 0; ch < nch; ++ch) s += (double)min(kBnChunk, B - ch * kBnChunk) * (double)ld(ch).x;
  const double mu = s / (double)B;
#pragma unroll 1
  for (int ch = 0; ch < nch; ++ch) {
    const float2 p = ld(ch);
    const double dlt = (double)p.x - mu;
    M2 += (double)p.y + (double)min(kBnChunk, B - ch * kBnChunk) * dlt * dlt;
  }
  mean = mu;
  var = M2 / (double)B;
}
template <class LD>
__device__ __forceinline__ void bn_bwd_sums_seq(LD ld, int B, double& s1, double& s2) {
  const int nch = (B + kBnChunk - 1) / kBnChunk;
  s1 = 0.0;
  s2 = 0.0;
#pragma unroll 1
  for (int ch = 0; ch < nch; ++ch) {
    const float2 p = ld(ch);
    s1 += (double)p.x;
    s2 += (double)p.y;
  }
}

// column col's coefficients and side outputs from its merged statistics
__device__ __forceinline__ void bn_fin_store(const BnFin& f, int col, double a, double b) {
  if (f.mode == 1) {  // a, b = mean, biased variance
    ((float2*)f.coef)[col] = bn_fwd_train_coef(a, b, (double)f.B, f.H, col, f.gamma, f.beta, f.rmean, f.rvar, f.save, true);
  } else {            // a, b = sum do, sum (y - mean) do
    const float invstd = f.save[f.H + col];
    f.dgamma[col] = (float)(b * invstd);
    f.dbeta[col] = (float)a;
    float cf[5];
    bn_bwd_coef(a, b, (double)f.B, f.train, f.H, col, f.save, f.gamma, f.beta, cf);
#pragma unroll
    for (int k = 0; k < 5; ++k) f.coef[(int64_t)k * f.H + col] = cf[k];
  }
}

// Called by EVERY thread of a workgroup after its partials of columns [col0, col0 + ncols) were
// stored with st_sc1_f2 (by any of its waves). Returns after the column block is finalised when this
// workgroup arrived last; otherwise returns at once. `flag`: one int of LDS the caller can spare.
// `stage` (optional, LDS the caller can spare, stage_cap float2): the last arriver first loads every
// chunk's partials of its columns there with ALL its threads (nch x ncols sc1 loads spread over the
// workgroup), then merges from LDS with one partial in registers at a time.
__device__ __forceinline__ void bn_fin_arrive(const BnFin& f, int block, int arrivals, int col0, int ncols,
                                              int* flag, float2* stage = nullptr, int stage_cap = 0) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x == 0)
    *flag = __hip_atomic_fetch_add((gi32_t*)(f.cnt + block), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (*flag != arrivals - 1) return;
  const int nch = (f.B + kBnChunk - 1) / kBnChunk;
  const int t = threadIdx.x;
  if (stage && nch * ncols <= stage_cap) {
#pragma unroll 1
    for (int i = t; i < nch * ncols; i += blockDim.x) {
      const int ch = i / ncols, c = col0 + i % ncols;
      stage[i] = c < f.H ? ld_sc1_f2(f.part + (int64_t)ch * f.H + c) : make_float2(0.f, 0.f);
    }
    __syncthreads();
    if (t < ncols && col0 + t < f.H) {
      auto ld = [&](int ch) { return stage[ch * ncols + t]; };
      double a, b;
      if (f.mode == 1) bn_merge_seq(ld, f.B, a, b);
      else bn_bwd_sums_seq(ld, f.B, a, b);
      bn_fin_store(f, col0 + t, a, b);
    }
  } else if (t < ncols && col0 + t < f.H) {
    const int col = col0 + t;
    auto ld = [&](int ch) { return ld_sc1_f2(f.part + (int64_t)ch * f.H + col); };
    double a, b;
    if (f.mode == 1) bn_merge_ld(ld, f.B, a, b);
    else bn_bwd_sums_ld(ld, f.B, a, b);
    bn_fin_store(f, col, a, b);
  }
  if (t == 0) __hip_atomic_store((gi32_t*)(f.cnt + block), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace gm2
