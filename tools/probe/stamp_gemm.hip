// Phase timestamps of the fp32-store GEMM kernel per workgroup (diagnostic probe, not part of
// libgm2): entry, first stage landed, main loop done, stores done. Prints the distribution of
// start skew, prologue, main loop and epilogue times for one shape (the hot path's own plan).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DGM2_STAMPS -I../../include
//        -I../../genome-minimizer-2_amd/csrc stamp_gemm.hip -o stamp_gemm
// Run:   ./stamp_gemm M N K pk qk      (pk/qk: operand K-major 1 / MN-major 0; random bf16 data)
#include "../../genome-minimizer-2_amd/csrc/gemm.hip"
#include "../../genome-minimizer-2_amd/csrc/options.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace gm2;

static void fill(bf16_t* d, size_t n, uint32_t seed) {
  std::vector<bf16_t> h(n);
  uint32_t x = seed * 2654435761u + 1;
  for (size_t i = 0; i < n; ++i) {
    x = x * 1664525u + 1013904223u;
    const float f = ((x >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f;  // uniform [-1, 1)
    uint32_t u;
    memcpy(&u, &f, 4);
    h[i] = (bf16_t)(u >> 16);
  }
  hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice);
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096, N = argc > 2 ? atoi(argv[2]) : 1024, K = argc > 3 ? atoi(argv[3]) : 1024;
  const int pk = argc > 4 ? atoi(argv[4]) : 1, qk = argc > 5 ? atoi(argv[5]) : 1;
  const int Mp = (M + 255) / 256 * 256, Np = (N + 255) / 256 * 256;
  bf16_t *P, *Q;
  float* C;
  hipMalloc(&P, (size_t)Mp * K * 2);
  hipMalloc(&Q, (size_t)Np * K * 2);
  hipMalloc(&C, (size_t)M * N * 4);
  fill(P, (size_t)Mp * K, 1);
  fill(Q, (size_t)Np * K, 2);
  GemmArgs<bf16_t> g{P, pk ? K : Mp, Q, qk ? K : Np, M, N, K, Mp, Np, 0, pk, qk};
  const GemmPlan pl = plan_gemm(g);
  for (int rep = 0; rep < 5; ++rep) launch_gemm_store<bf16_t>(g, pl.splits, C, nullptr, 0, N, 0, nullptr, nullptr);
  hipDeviceSynchronize();
  const int tiles = (Mp / pl.tile) * (Np / pl.tile) * pl.splits;
  std::vector<unsigned long long> st((size_t)16384 * 8);
  hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamp), st.size() * 8);
  unsigned long long t0 = ~0ull, tend = 0;
  for (int b = 0; b < tiles; ++b) {
    t0 = std::min(t0, st[b * 8]);
    tend = std::max(tend, st[b * 8 + 3]);
  }
  std::vector<double> skew, pro, loop, epi;
  for (int b = 0; b < tiles; ++b) {
    const unsigned long long* s = &st[b * 8];
    skew.push_back((s[0] - t0) * 0.01);
    pro.push_back((s[1] - s[0]) * 0.01);
    loop.push_back((s[2] - s[1]) * 0.01);
    epi.push_back((s[3] - s[2]) * 0.01);
  }
  auto pr = [](const char* n, std::vector<double> v) {
    std::sort(v.begin(), v.end());
    printf("%-8s min %7.2f  med %7.2f  p90 %7.2f  max %7.2f us\n", n, v[0], v[v.size() / 2], v[v.size() * 9 / 10], v.back());
  };
  printf("M=%d N=%d K=%d pk=%d qk=%d tile=%d splits=%d tiles=%d: first start -> last end %.2f us\n", M, N, K, pk, qk,
         pl.tile, pl.splits, tiles, (tend - t0) * 0.01);
  pr("skew", skew);
  pr("prologue", pro);
  pr("mainloop", loop);
  pr("epilogue", epi);
  return 0;
}
