// Phase timestamps of the fp32-store GEMM kernel per workgroup (diagnostic probe, not part of
// libgm2): entry, first stage landed, main loop done, stores done. Prints the distribution of
// start skew, prologue, main loop and epilogue times for the hidden-layer shape.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DGM2_STAMPS -I../../include
//        -I../../genome-minimizer-2_amd/csrc stamp_gemm.hip -o stamp_gemm
#include "../../genome-minimizer-2_amd/csrc/gemm.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

using namespace gm2;

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096, N = argc > 2 ? atoi(argv[2]) : 1024, K = argc > 3 ? atoi(argv[3]) : 1024;
  bf16_t *P, *Q;
  float* C;
  hipMalloc(&P, (size_t)M * K * 2);
  hipMalloc(&Q, (size_t)N * K * 2);
  hipMalloc(&C, (size_t)M * N * 4);
  hipMemset(P, 0, (size_t)M * K * 2);
  hipMemset(Q, 0, (size_t)N * K * 2);
  GemmArgs<bf16_t> g{P, K, Q, K, M, N, K, M, N, 0, 1, 1};
  for (int rep = 0; rep < 5; ++rep) launch_gemm_store<bf16_t>(g, 1, C, nullptr, 0, N, 0, nullptr, nullptr);
  hipDeviceSynchronize();
  const int tiles = (M / 128) * (N / 128);
  std::vector<unsigned long long> st((size_t)16384 * 4);
  hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamp), st.size() * 8);
  unsigned long long t0 = ~0ull, tend = 0;
  for (int b = 0; b < tiles; ++b) {
    t0 = std::min(t0, st[b * 4]);
    tend = std::max(tend, st[b * 4 + 3]);
  }
  std::vector<double> skew, pro, loop, epi;
  for (int b = 0; b < tiles; ++b) {
    const unsigned long long* s = &st[b * 4];
    skew.push_back((s[0] - t0) * 0.01);
    pro.push_back((s[1] - s[0]) * 0.01);
    loop.push_back((s[2] - s[1]) * 0.01);
    epi.push_back((s[3] - s[2]) * 0.01);
  }
  auto pr = [](const char* n, std::vector<double> v) {
    std::sort(v.begin(), v.end());
    printf("%-8s min %7.2f  med %7.2f  p90 %7.2f  max %7.2f us\n", n, v[0], v[v.size() / 2], v[v.size() * 9 / 10], v.back());
  };
  printf("M=%d N=%d K=%d tiles=%d: first start -> last end %.2f us\n", M, N, K, tiles, (tend - t0) * 0.01);
  pr("skew", skew);
  pr("prologue", pro);
  pr("mainloop", loop);
  pr("epilogue", epi);
  return 0;
}
