// BatchNorm1d finalisation arithmetic (training/model.py:66-86, nn.BatchNorm1d train mode) shared by
// the apply kernels (kernels.hip): the fp64 chunk merges of the per-128-row partials and the
// per-column coefficients.
//
// Statistics arrive as per-128-row-chunk partials part[chunk][H] (float2):
//   forward : (chunk mean, chunk M2) of the pre-BN output y
//   backward: (sum do, sum (y - mean) do), do = dA * [bn output > 0]
// (Round 4 also tried finalising them in the LAST-arriving workgroup of the kernel that produced the
// statistics, so the apply passes would only read a table: the producers grew 5-25 us each and the
// step +40 us, profiles/r04_bn_fin_ab.txt; removed.)
#pragma once
#include "gm2_common.hpp"

namespace gm2 {

constexpr double kBnEps = 1e-5;       // nn.BatchNorm1d default eps
constexpr double kBnMomentum = 0.1;   // nn.BatchNorm1d default momentum
constexpr int kBnChunk = 128;         // rows per partial-statistics chunk (= kBnRowChunk)

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

}  // namespace gm2
