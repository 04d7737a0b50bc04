// Launch time of the one-pass weight-gradient GEMM (launch_gemm_sq: fp32 store + per-tile sums of
// squares) alone on the chip, per grid mode (diagnostic probe, not part of libgm2):
//   mode 0 one workgroup per tile, 1 capped grid (GM2_OPT_GRID_CAP bit 2). Random bf16 operands. With -DGM2_STAMPS it also prints the phase
//   distribution per workgroup (entry, main loop done, stores done).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 [-DGM2_STAMPS] -I../../include
//        -I../../genome-minimizer-2_amd/csrc time_sq.hip -o time_sq
// Run:   ./time_sq M N K pk qk mode [reps]
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
    const float f = ((x >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f;
    uint32_t u;
    memcpy(&u, &f, 4);
    h[i] = (bf16_t)(u >> 16);
  }
  hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice);
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 1024, N = argc > 2 ? atoi(argv[2]) : 55040, K = argc > 3 ? atoi(argv[3]) : 4096;
  const int pk = argc > 4 ? atoi(argv[4]) : 1, qk = argc > 5 ? atoi(argv[5]) : 0, mode = argc > 6 ? atoi(argv[6]) : 0;
  const int reps = argc > 7 ? atoi(argv[7]) : 20;
  const int Mp = (M + 255) / 256 * 256, Np = (N + 255) / 256 * 256;
  bf16_t *P, *Q;
  float* C;
  double* sq;
  hipMalloc(&P, (size_t)Mp * K * 2);
  hipMalloc(&Q, (size_t)Np * K * 2);
  hipMalloc(&C, (size_t)M * N * 4);
  hipMalloc(&sq, (size_t)(Mp / 256) * (Np / 256) * 8);
  fill(P, (size_t)Mp * K, 1);
  fill(Q, (size_t)Np * K, 2);
  GemmArgs<bf16_t> g{P, pk ? K : Mp, Q, qk ? K : Np, M, N, K, Mp, Np, 0, pk, qk};
  Options o = default_options();
  o.grid_cap = mode == 1 ? 2 : 0;
  OptionScope scope(o);
  auto run = [&] { launch_gemm_sq<bf16_t>(g, C, N, sq, nullptr, false); };
  for (int r = 0; r < 3; ++r) run();
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, nullptr);
  for (int r = 0; r < reps; ++r) run();
  hipEventRecord(e1, nullptr);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  printf("M=%d N=%d K=%d pk=%d qk=%d mode=%d: %.1f us per launch (%d launches)\n", M, N, K, pk, qk, mode,
         1000.f * ms / reps, reps);
#ifdef GM2_STAMPS
  const int blocks = std::min(16384, (Mp / 256) * (Np / 256) * 2);
  std::vector<unsigned long long> st((size_t)16384 * 8);
  hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamp), st.size() * 8);
  unsigned long long t0 = ~0ull;
  for (int b = 0; b < blocks; ++b)
    if (st[b * 8]) t0 = std::min(t0, st[b * 8]);
  // per workgroup: start, main loop done (stamp 2), end (stamp 3; 0 for a part that did not store)
  std::vector<double> start, loop, end;
  for (int b = 0; b < blocks; ++b) {
    const unsigned long long* s = &st[b * 8];
    if (!s[0] || s[0] < t0) continue;
    start.push_back((s[0] - t0) * 0.01);
    if (s[2] > s[0]) loop.push_back((s[2] - s[0]) * 0.01);
    if (s[3] > s[0]) end.push_back((s[3] - t0) * 0.01);
  }
  auto pr = [](const char* n, std::vector<double> v) {
    if (v.empty()) return;
    std::sort(v.begin(), v.end());
    printf("%-10s n %5zu  min %7.2f  med %7.2f  p90 %7.2f  max %7.2f us\n", n, v.size(), v[0], v[v.size() / 2],
           v[v.size() * 9 / 10], v.back());
  };
  pr("start", start);
  pr("to-loop", loop);
  pr("end", end);
#endif
  return 0;
}
