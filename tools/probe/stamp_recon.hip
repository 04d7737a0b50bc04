// Phase timestamps of the output-layer loss kernel (k_gemm_recon_loss) per workgroup (diagnostic
// probe, not part of libgm2): entry, first K-tile landed, main loop done, element loop done,
// dL / column-sum stores landed. Prints the distribution of each phase for the C2 shape.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DGM2_STAMPS -I../../include
//        -I../../genome-minimizer-2_amd/csrc stamp_recon.hip -o stamp_recon
// Run:   ./stamp_recon [G B H]      (random bf16 operands, random target bits, v0 scalars)
#include "../../genome-minimizer-2_amd/csrc/gemm.hip"
#include "../../genome-minimizer-2_amd/csrc/options.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace gm2;

static void fill(bf16_t* d, size_t n, uint32_t seed, float scale) {
  std::vector<bf16_t> h(n);
  uint32_t x = seed * 2654435761u + 1;
  for (size_t i = 0; i < n; ++i) {
    x = x * 1664525u + 1013904223u;
    const float f = (((x >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f) * scale;
    uint32_t u;
    memcpy(&u, &f, 4);
    h[i] = (bf16_t)(u >> 16);
  }
  hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice);
}

int main(int argc, char** argv) {
  const int G = argc > 1 ? atoi(argv[1]) : 55039, B = argc > 2 ? atoi(argv[2]) : 4096, H = argc > 3 ? atoi(argv[3]) : 1024;
  const int Gp = (G + 255) / 256 * 256, Bp = (B + 255) / 256 * 256;
  const int64_t ldx = Gp / 32, ldd = Gp;
  bf16_t *W, *A, *dL;
  float *bias, *scal, *loss, *col;
  uint32_t* X;
  hipMalloc(&W, (size_t)Gp * H * 2);
  hipMalloc(&A, (size_t)Bp * H * 2);
  hipMalloc(&dL, (size_t)Bp * ldd * 2);
  hipMalloc(&bias, (size_t)Gp * 4);
  hipMalloc(&scal, 64 * 4);
  hipMalloc(&loss, (size_t)(Gp / 128) * (Bp / 128) * 2 * 4);
  hipMalloc(&col, (size_t)(Bp / 128) * Gp * 4);
  hipMalloc(&X, (size_t)Bp * ldx * 4);
  fill(W, (size_t)Gp * H, 1, 0.05f);
  fill(A, (size_t)Bp * H, 2, 1.0f);
  hipMemset(bias, 0, (size_t)Gp * 4);
  hipMemset(scal, 0, 64 * 4);
  {
    std::vector<uint32_t> h((size_t)Bp * ldx);
    uint32_t x = 7;
    for (auto& w : h) {
      x = x * 1664525u + 1013904223u;
      w = x;
    }
    hipMemcpy(X, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  }
  GemmArgs<bf16_t> g{W, H, A, H, G, B, H, Gp, Bp, 0, 1, 1};
  for (int rep = 0; rep < 5; ++rep)
    launch_gemm_recon_loss<bf16_t>(g, bias, X, ldx, 1, scal, dL, ldd, loss, col, Gp, nullptr);
  hipDeviceSynchronize();
  const int tiles = gemm_recon_grid_blocks<bf16_t>(g);
  std::vector<unsigned long long> st((size_t)16384 * 8);
  hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamp), st.size() * 8);
  unsigned long long t0 = ~0ull, tend = 0;
  for (int b = 0; b < tiles; ++b) {
    t0 = std::min(t0, st[b * 8]);
    tend = std::max(tend, st[b * 8 + 3]);
  }
  std::vector<double> skew, pro, loop, elem, store, total;
  for (int b = 0; b < tiles; ++b) {
    const unsigned long long* s = &st[b * 8];
    skew.push_back((s[0] - t0) * 0.01);
    pro.push_back((s[1] - s[0]) * 0.01);
    loop.push_back((s[2] - s[1]) * 0.01);
    elem.push_back((s[4] - s[2]) * 0.01);
    store.push_back((s[3] - s[4]) * 0.01);
    total.push_back((s[3] - s[0]) * 0.01);
  }
  auto pr = [](const char* n, std::vector<double> v) {
    std::sort(v.begin(), v.end());
    double m = 0;
    for (double x : v) m += x;
    printf("%-9s mean %7.2f  min %7.2f  med %7.2f  p90 %7.2f  max %7.2f us\n", n, m / v.size(), v[0], v[v.size() / 2],
           v[v.size() * 9 / 10], v.back());
  };
  printf("G=%d B=%d H=%d tiles=%d: first start -> last end %.2f us\n", G, B, H, tiles, (tend - t0) * 0.01);
  pr("skew", skew);
  pr("prologue", pro);
  pr("mainloop", loop);
  pr("elements", elem);
  pr("stores", store);
  pr("total", total);
  // time per launch without stamps' own cost is the bench's number; this is the phase split
  return 0;
}
