// MFMA GEMM for the VAE hot path: C[M,N] = sum_k P[m,k] * Q[n,k]  ("NT": both operands
// K-contiguous, the layout the 16x16 MFMA fragments read with one ds_read_b128 per lane).
//
//  * T = bf16_t : v_mfma_f32_16x16x32_bf16 (training fast path, fp32 accumulate)
//  * T = float  : v_mfma_f32_16x16x4_f32   (exact-f32 path: sampling decode + parity training)
//
// Block tile 128x128, 4 waves (2x2), each wave 64x64 = 4x4 MFMA tiles; one K-step = one
// 128-byte row chunk per operand row (64 bf16 / 32 f32). Operands are staged HBM->LDS with
// global_load_lds_dwordx4 (no VGPR round trip) into a 2-stage ring; the LDS image is
// XOR-swizzled (chunk ^= (row>>1)&7) by permuting the per-lane SOURCE address, which makes the
// 16-lane ds_read_b128 groups conflict-free.
//
// Contract (checked on the host in api.cpp): every operand buffer has >= roundup(M|N,128)
// rows, K is a multiple of 64, pads are zero. Split-K over blockIdx.z.
#include "gm2_common.hpp"
#include "gm2_kernels.hpp"

#include <utility>
#include <vector>

namespace gm2 {

namespace {

constexpr int kThreads = 256;
constexpr int kStageBytes = 2 * kTile * 128;  // A + B, 16 KiB each
constexpr int kLdsBytes = 2 * kStageBytes;    // double buffered: 64 KiB

typedef __attribute__((address_space(3))) void lds_void;

template <typename T>
__device__ __forceinline__ void stage_tile(const T* __restrict__ P, int64_t ldp, int row0, int k0,
                                           char* lds, int wid, int lane) {
  // 128 rows x 128 B = 1024 16-byte chunks; 256 threads -> 4 glds per thread.
  // wave instruction j covers chunks [j*256 + wid*64, +64): LDS dest is lane-linear.
  constexpr int EPC = 16 / sizeof(T);  // elements per 16-byte chunk
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = j * 256 + wid * 64 + lane;
    const int row = i >> 3;
    const int cs = i & 7;
    const int c = cs ^ ((row >> 1) & 7);
    const T* src = P + (int64_t)(row0 + row) * ldp + k0 + c * EPC;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds + (j * 256 + wid * 64) * 16),
                                     16, 0, 0);
  }
}

__device__ __forceinline__ int frag_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

// Main loop. acc[mi][ni] holds rows wm*64+mi*16+4*(lane>>4)+j, cols wn*64+ni*16+(lane&15).
template <typename T>
__device__ __forceinline__ void gemm_mainloop(const T* __restrict__ P, int64_t ldp,
                                              const T* __restrict__ Q, int64_t ldq, int m0, int n0,
                                              int kbeg, int nk, char* smem, f32x4 (&acc)[4][4]) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  constexpr int KT = E<T>::KT;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nk <= 0) return;

  stage_tile<T>(P, ldp, m0, kbeg, smem, wid, lane);
  stage_tile<T>(Q, ldq, n0, kbeg, smem + kTile * 128, wid, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * kStageBytes;
    if (kt + 1 < nk) {
      char* nxt = smem + ((kt + 1) & 1) * kStageBytes;
      const int kn = kbeg + (kt + 1) * KT;
      stage_tile<T>(P, ldp, m0, kn, nxt, wid, lane);
      stage_tile<T>(Q, ldq, n0, kn, nxt + kTile * 128, wid, lane);
    }
    const char* sA = cur;
    const char* sB = cur + kTile * 128;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = s * 4 + (lane >> 4);
      if constexpr (sizeof(T) == 2) {
        bf16x8 a[4], b[4];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
          a[mi] = *(const bf16x8*)(sA + frag_off(wm * 64 + mi * 16 + (lane & 15), c));
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          b[ni] = *(const bf16x8*)(sB + frag_off(wn * 64 + ni * 16 + (lane & 15), c));
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
      } else {
        f32x4 a[4], b[4];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
          a[mi] = *(const f32x4*)(sA + frag_off(wm * 64 + mi * 16 + (lane & 15), c));
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          b[ni] = *(const f32x4*)(sB + frag_off(wn * 64 + ni * 16 + (lane & 15), c));
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mi][j], b[ni][j], acc[mi][ni], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// Epilogue 1: fp32 store. Rows m < msplit go to C0, rows >= msplit to C1 (row m - msplit); the
// split-K slice z writes slab z (C0 + z*slab). Optional per-column bias.
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kThreads, 2) void k_gemm_store(GemmArgs<T> g, float* __restrict__ C0,
                                                          float* __restrict__ C1, int msplit,
                                                          int64_t ldc, int64_t slab,
                                                          const float* __restrict__ bias) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n0 = blockIdx.x * kTile, m0 = blockIdx.y * kTile;
  const int kbeg = blockIdx.z * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  const int nk = (kend - kbeg) / E<T>::KT;
  f32x4 acc[4][4];
  gemm_mainloop<T>(g.P, g.ldp, g.Q, g.ldq, m0, n0, kbeg, nk, smem, acc);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wm = wid >> 1, wn = wid & 1;
  float* Cz = C0 + (int64_t)blockIdx.z * slab;
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int n = n0 + wn * 64 + ni * 16 + (lane & 15);
    if (n >= g.N) continue;
    const float bn = bias ? bias[n] : 0.f;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + wm * 64 + mi * 16 + 4 * (lane >> 4) + j;
        if (m >= g.M) continue;
        const float v = acc[mi][ni][j] + bn;
        if (m < msplit) Cz[(int64_t)m * ldc + n] = v;
        else C1[(int64_t)(m - msplit) * ldc + n] = v;
      }
  }
}

// ---------------------------------------------------------------------------------------------
// Epilogue 2: decoder output layer + reconstruction loss (loss_components.py:49-50 BCE(sum),
// :111-115 gene abundance) and, in training, dL/dlogit exactly as autograd composes
// Sigmoid->BCE: dp = (p-x)/max((1-p)p, 1e-12) + w*gamma ; dl = dp*(1-p)*p.
// (sign(colsum p) == 1 wherever p > 0, and dl == 0 wherever p == 0: no batch-wide pass needed.)
// Writes dL [m][ldd] and dL^T [n][lddt] (both T, zero outside the valid MxN box), the per-block
// sums of BCE and p (loss_part[blk*2 + {0,1}]) and the per-(m-tile, n) column sums of dl.
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kThreads, 2) void k_gemm_recon_loss(
    GemmArgs<T> g, const float* __restrict__ bias, const T* __restrict__ X, int64_t ldx,
    int with_grad, const float* __restrict__ scal, T* __restrict__ dL, int64_t ldd,
    T* __restrict__ dLT, int64_t lddt, float* __restrict__ loss_part, float* __restrict__ colpart,
    int64_t ldcol) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n0 = blockIdx.x * kTile, m0 = blockIdx.y * kTile;
  f32x4 acc[4][4];
  gemm_mainloop<T>(g.P, g.ldp, g.Q, g.ldq, m0, n0, 0, g.K / E<T>::KT, smem, acc);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wm = wid >> 1, wn = wid & 1;
  const float wgam = scal[kScalWGamma];
  float bce = 0.f, psum = 0.f;
  float csum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int n = n0 + wn * 64 + ni * 16 + (lane & 15);
    const bool nok = n < g.N;
    const float bn = nok ? bias[n] : 0.f;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int mb = m0 + wm * 64 + mi * 16 + 4 * (lane >> 4);
      float dl4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = mb + j;
        float dl = 0.f;
        if (nok && m < g.M) {
          const float l = acc[mi][ni][j] + bn;
          const float p = 1.0f / (1.0f + expf(-l));
          const float x = E<T>::ld(X + (int64_t)m * ldx + n);
          // BCE element (x in {0,1}): (x-1)*max(log1p(-p),-100) - x*max(log(p),-100)
          const float e = x != 0.f ? -fmaxf(logf(p), -100.f) : -fmaxf(log1pf(-p), -100.f);
          bce += e;
          psum += p;
          const float omp = 1.0f - p;
          const float dp = (p - x) / fmaxf(omp * p, 1e-12f) + wgam;
          dl = dp * omp * p;
          csum[ni] += dl;
        }
        dl4[j] = dl;
      }
      if (with_grad) {
        if (mb < g.Mp) {  // padded rows are written (as zeros) so K-pads stay zero downstream
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (n < g.Np) dL[(int64_t)(mb + j) * ldd + n] = E<T>::cvt(dl4[j]);
          if (n < g.Np) {
            if constexpr (sizeof(T) == 2) {
              uint2 pk;
              pk.x = (uint32_t)f2bf(dl4[0]) | ((uint32_t)f2bf(dl4[1]) << 16);
              pk.y = (uint32_t)f2bf(dl4[2]) | ((uint32_t)f2bf(dl4[3]) << 16);
              *(uint2*)(dLT + (int64_t)n * lddt + mb) = pk;
            } else {
              *(f32x4*)(dLT + (int64_t)n * lddt + mb) = f32x4{dl4[0], dl4[1], dl4[2], dl4[3]};
            }
          }
        }
      }
    }
  }
  // block reductions: BCE, sum(p) -> loss_part; column sums of dl over this block's 128 rows
  // the main loop ended on a barrier: reuse the staging LDS for the reductions (one LDS object)
  float(*red)[4] = (float(*)[4])smem;
  float(*colred)[128] = (float(*)[128])(smem + 64);
  bce = wave_sum(bce);
  psum = wave_sum(psum);
  if (lane == 0) { red[0][wid] = bce; red[1][wid] = psum; }
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    float v = csum[ni];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (lane < 16) colred[wm][wn * 64 + ni * 16 + lane] = v;
  }
  __syncthreads();
  const int blk = blockIdx.y * gridDim.x + blockIdx.x;
  if (threadIdx.x == 0) {
    loss_part[blk * 2 + 0] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    loss_part[blk * 2 + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
  if (with_grad && threadIdx.x < 128) {
    const int n = n0 + threadIdx.x;
    if (n < g.N) colpart[(int64_t)blockIdx.y * ldcol + n] = colred[0][threadIdx.x] + colred[1][threadIdx.x];
  }
}

// ---------------------------------------------------------------------------------------------
// Epilogue 3: sampling output layer. mask = logit > 0x33C00000 (== sigmoid_fp32 > 0.5,
// extras.py:200-201); optional probabilities p = sigmoid(logit) (extras.py:198).
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kThreads, 2) void k_gemm_mask(GemmArgs<T> g, const float* __restrict__ bias,
                                                         uint8_t* __restrict__ mask, int64_t ldm,
                                                         float* __restrict__ probs, int64_t ldpr) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n0 = blockIdx.x * kTile, m0 = blockIdx.y * kTile;
  f32x4 acc[4][4];
  gemm_mainloop<T>(g.P, g.ldp, g.Q, g.ldq, m0, n0, 0, g.K / E<T>::KT, smem, acc);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wm = wid >> 1, wn = wid & 1;
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int n = n0 + wn * 64 + ni * 16 + (lane & 15);
    if (n >= g.N) continue;
    const float bn = bias[n];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + wm * 64 + mi * 16 + 4 * (lane >> 4) + j;
        if (m >= g.M) continue;
        const float l = acc[mi][ni][j] + bn;
        mask[(int64_t)m * ldm + n] = l > kMaskLogitThreshold ? 1 : 0;
        if (probs) probs[(int64_t)m * ldpr + n] = 1.0f / (1.0f + expf(-l));
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
  size_t used = 0;
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
  for (size_t i = 0; i < t.used; ++i) {
    hipError_t e = hipEventSynchronize(t.ev[i].second);
    if (e != hipSuccess) throw Gm2Error("timing: %s", hipGetErrorString(e));
    float ms = 0.f;
    e = hipEventElapsedTime(&ms, t.ev[i].first, t.ev[i].second);
    if (e != hipSuccess) throw Gm2Error("timing: %s", hipGetErrorString(e));
    tot += ms;
  }
  *total_ms = tot;
  *launches = (int64_t)t.used;
  t.classes = 0;
  t.used = 0;
}

TimedLaunch::TimedLaunch(int cls, hipStream_t st) : idx(-1), s(st) {
  TimingState& t = tstate();
  if (!(t.classes & cls)) return;
  if (t.used == t.ev.size()) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) throw Gm2Error("hipEventCreate");
    t.ev.push_back({a, b});
  }
  idx = (int)t.used++;
  if (hipEventRecord(t.ev[idx].first, s) != hipSuccess) throw Gm2Error("hipEventRecord");
}

TimedLaunch::~TimedLaunch() {
  if (idx >= 0) (void)hipEventRecord(tstate().ev[idx].second, s);
}

// ------------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------------
template <typename T>
static void check_gemm(const GemmArgs<T>& g) {
  if (g.K % kKPad || g.Mp % kTile || g.Np % kTile || g.M > g.Mp || g.N > g.Np || g.M <= 0 || g.N <= 0)
    throw Gm2Error("gemm: bad dims M=%d N=%d K=%d Mp=%d Np=%d", g.M, g.N, g.K, g.Mp, g.Np);
  if (g.ldp < g.K || g.ldq < g.K) throw Gm2Error("gemm: ld < K");
  if (((uintptr_t)g.P | (uintptr_t)g.Q) & 15) throw Gm2Error("gemm: operands not 16-B aligned");
  if ((g.ldp * sizeof(T)) % 16 || (g.ldq * sizeof(T)) % 16) throw Gm2Error("gemm: ld not 16-B multiple");
}

template <typename T>
int launch_gemm_store(const GemmArgs<T>& g, int splits, float* C0, float* C1, int msplit, int64_t ldc,
                      int64_t slab, const float* bias, hipStream_t s) {
  check_gemm(g);
  GemmArgs<T> a = g;
  const int kt = E<T>::KT;
  const int nkt = g.K / kt;
  splits = std::max(1, std::min(splits, nkt));
  a.k_per_split = (int)(round_up(nkt, splits) / splits) * kt;
  splits = (int)((g.K + a.k_per_split - 1) / a.k_per_split);
  dim3 grid(g.Np / kTile, g.Mp / kTile, splits);
  TimedLaunch tl(kKcGemmStore, s);
  hipLaunchKernelGGL(k_gemm_store<T>, grid, dim3(kThreads), kLdsBytes, s, a, C0, C1 ? C1 : C0,
                     C1 ? msplit : (1 << 30), ldc, slab, bias);
  GM2_CHECK_LAUNCH();
  return splits;
}

template <typename T>
int gemm_recon_grid_blocks(const GemmArgs<T>& g) { return (g.Np / kTile) * (g.Mp / kTile); }

template <typename T>
void launch_gemm_recon_loss(const GemmArgs<T>& g, const float* bias, const T* X, int64_t ldx, int with_grad,
                            const float* scal, T* dL, int64_t ldd, T* dLT, int64_t lddt, float* loss_part,
                            float* colpart, int64_t ldcol, hipStream_t s) {
  check_gemm(g);
  dim3 grid(g.Np / kTile, g.Mp / kTile, 1);
  TimedLaunch tl(kKcReconLoss, s);
  hipLaunchKernelGGL(k_gemm_recon_loss<T>, grid, dim3(kThreads), kLdsBytes, s, g, bias, X, ldx, with_grad, scal,
                     dL, ldd, dLT, lddt, loss_part, colpart, ldcol);
  GM2_CHECK_LAUNCH();
}

template <typename T>
void launch_gemm_mask(const GemmArgs<T>& g, const float* bias, uint8_t* mask, int64_t ldm, float* probs,
                      int64_t ldpr, hipStream_t s) {
  check_gemm(g);
  dim3 grid(g.Np / kTile, g.Mp / kTile, 1);
  TimedLaunch tl(kKcMask, s);
  hipLaunchKernelGGL(k_gemm_mask<T>, grid, dim3(kThreads), kLdsBytes, s, g, bias, mask, ldm, probs, ldpr);
  GM2_CHECK_LAUNCH();
}

template int launch_gemm_store<float>(const GemmArgs<float>&, int, float*, float*, int, int64_t, int64_t,
                                       const float*, hipStream_t);
template int launch_gemm_store<bf16_t>(const GemmArgs<bf16_t>&, int, float*, float*, int, int64_t, int64_t,
                                        const float*, hipStream_t);
template void launch_gemm_recon_loss<float>(const GemmArgs<float>&, const float*, const float*, int64_t, int,
                                            const float*, float*, int64_t, float*, int64_t, float*, float*,
                                            int64_t, hipStream_t);
template void launch_gemm_recon_loss<bf16_t>(const GemmArgs<bf16_t>&, const float*, const bf16_t*, int64_t, int,
                                             const float*, bf16_t*, int64_t, bf16_t*, int64_t, float*, float*,
                                             int64_t, hipStream_t);
template void launch_gemm_mask<float>(const GemmArgs<float>&, const float*, uint8_t*, int64_t, float*, int64_t,
                                      hipStream_t);
template int gemm_recon_grid_blocks<float>(const GemmArgs<float>&);
template int gemm_recon_grid_blocks<bf16_t>(const GemmArgs<bf16_t>&);

}  // namespace gm2
