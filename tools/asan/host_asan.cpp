// AddressSanitizer driver of libgm2's host-side logic (race detection / sanitizers).
// Built by `build_native.py --variant asan`: every csrc/*.hip compiled -DGM2_DEBUG with ASan on the
// HOST code only (-Xarch_host -fsanitize=address), linked with this file into one executable. It
// needs no GPU and launches no kernel: it drives the C-ABI entry points whose work is host
// arithmetic -- dims and parameter offsets, the workspace layout (gm2_debug_check_layout: alignment,
// overlap, bounds of every region), resident-operand layouts, gradient buckets, the option tables
// (every key, valid and invalid values, process defaults vs per-workspace state), and the error
// paths of every entry point given null / inconsistent arguments or an unknown workspace -- so any
// heap / stack / global overflow or use-after-free in that code aborts the run with an ASan report.
// Exit code 0 = every check passed and ASan saw nothing. tests/test_asan_cpu.py runs it.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gm2.h"
#include "../../include/gm2_debug.h"

static int g_fail = 0;
#define CHECK(c, ...)                                     \
  do {                                                    \
    if (!(c)) {                                           \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                  \
      std::fprintf(stderr, "\n");                         \
      ++g_fail;                                           \
    }                                                     \
  } while (0)

// a call that must fail with a message containing `what`
static void expect_error(int rc, const char* what, const char* ctx) {
  CHECK(rc != 0, "%s: expected an error", ctx);
  const char* e = gm2_last_error();
  CHECK(e && std::strstr(e, what), "%s: error '%s' lacks '%s'", ctx, e ? e : "(null)", what);
}

static void dims_and_layouts() {
  const int64_t Gs[] = {1, 2, 127, 128, 129, 255, 256, 257, 20000, 55039};
  const int64_t Hs[] = {128, 256, 512, 1024};
  const int64_t Ls[] = {1, 2, 4, 8, 16, 32, 64, 128, 256};
  const int64_t Bs[] = {1, 2, 3, 63, 64, 127, 128, 129, 4096, 4097};
  int64_t checked = 0;
  for (int64_t G : Gs)
    for (int64_t H : Hs)
      for (int64_t L : Ls)
        for (int64_t B : Bs) {
          if (G * H > (int64_t)64 << 20 && B > 256 && H != 1024) continue;  // keep the sweep short
          gm2_dims d{G, H, L, B};
          int64_t n = 0;
          CHECK(gm2_param_count(&d, &n) == 0, "param_count %s", gm2_last_error());
          std::vector<int64_t> off(GM2_NUM_PARAMS + 1, -1);
          CHECK(gm2_param_offsets(&d, off.data()) == 0, "param_offsets");
          CHECK(off[0] == 0 && off[GM2_NUM_PARAMS] == n, "offsets span [0, %lld)", (long long)n);
          for (int i = 0; i < GM2_NUM_PARAMS; ++i) CHECK(off[i] < off[i + 1], "offsets ascend at %d", i);
          std::vector<int64_t> lh(2 * GM2_GRAD_BUCKETS, -1);
          CHECK(gm2_grad_bucket_bounds(&d, lh.data()) == 0, "bucket bounds");
          for (int b = 0; b < GM2_GRAD_BUCKETS; ++b)
            CHECK(0 <= lh[2 * b] && lh[2 * b] <= lh[2 * b + 1] && lh[2 * b + 1] <= n, "bucket %d in range", b);
          for (int prec : {GM2_F32, GM2_BF16}) {
            size_t bytes = 0;
            CHECK(gm2_workspace_size(&d, prec, &bytes) == 0, "workspace_size %s", gm2_last_error());
            int64_t nreg = 0, total = 0;
            const int rc = gm2_debug_check_layout(&d, prec, &nreg, &total);
            CHECK(rc == 0, "layout G=%lld H=%lld L=%lld B=%lld prec=%d: %s", (long long)G, (long long)H,
                  (long long)L, (long long)B, prec, gm2_last_error());
            CHECK((size_t)total == bytes && nreg > 50, "layout total %lld vs size %zu, %lld regions",
                  (long long)total, bytes, (long long)nreg);
            ++checked;
          }
        }
  std::printf("layouts checked: %lld\n", (long long)checked);
  // bad dims
  gm2_dims bad[] = {{0, 128, 8, 8}, {10, 100, 8, 8}, {10, 128, 3, 8}, {10, 128, 8, 0}, {-5, 128, 8, 8}};
  size_t bytes = 0;
  for (auto& d : bad) CHECK(gm2_workspace_size(&d, GM2_BF16, &bytes) != 0, "bad dims accepted");
  expect_error(gm2_workspace_size(nullptr, GM2_BF16, &bytes), "null dims", "null dims");
  gm2_dims d{100, 128, 8, 16};
  expect_error(gm2_workspace_size(&d, 7, &bytes), "precision", "bad precision");
  // resident layouts
  for (int64_t S : {1, 2, 63, 64, 10000})
    for (int64_t G : {1, 255, 256, 20000, 55039})
      for (int prec : {GM2_F32, GM2_BF16}) {
        int64_t ld = 0, ldb = 0, rows = 0;
        size_t nb = 0, nbb = 0;
        CHECK(gm2_resident_layout(S, G, prec, &ld, &ldb, &rows, &nb, &nbb) == 0, "resident layout %s",
              gm2_last_error());
        CHECK(ld >= G && ld % 256 == 0 && ldb * 32 == ld && rows >= S + 1 && rows % 64 == 0, "resident shape");
        CHECK(nb == (size_t)(rows * ld * (prec == GM2_F32 ? 4 : 2)) && nbb == (size_t)(rows * ldb * 4),
              "resident bytes");
      }
  for (int64_t G : {1, 8, 9, 127, 128, 55039}) CHECK(gm2_packed_row_bytes(G) >= (G + 7) / 8, "packed row bytes");
}

static const int kKeys[] = {GM2_OPT_GEMM_PP,      GM2_OPT_SIDE_STREAM,  GM2_OPT_RECON_TILE,        GM2_OPT_SMALL_SPLIT,
                            GM2_OPT_BN_EPILOGUE,  GM2_OPT_SMALL_WAVES,  GM2_OPT_INPUT_CHUNKS,      GM2_OPT_GRID_CAP,
                            GM2_OPT_SYNC_BN,      GM2_OPT_DEFER_OUTPUT_ADAM, GM2_OPT_GRAD_BUCKETS, GM2_OPT_SAMPLE_SPLIT,
                            GM2_OPT_SAMPLE_SINGLE, GM2_OPT_SAMPLE_BAND_CAP, GM2_OPT_SAMPLE_SINGLE_BOUND};

static void options() {
  std::vector<int> saved;
  for (int k : kKeys) {
    int v = -99;
    CHECK(gm2_get_option(k, &v) == 0, "get option %d", k);
    saved.push_back(v);
  }
  // every key: a sweep of values; accepted ones read back as set (or clamped / booleanised)
  const int probe[] = {-100000, -2, -1, 0, 1, 2, 3, 4, 5, 7, 8, 9, 16, 17, 64, 128, 256, 4096, 4097, 1 << 30};
  int accepted = 0, rejected = 0;
  for (int k : kKeys)
    for (int v : probe) {
      int before = 0;
      gm2_get_option(k, &before);
      if (gm2_set_option(k, v) == 0) {
        int got = -12345;
        CHECK(gm2_get_option(k, &got) == 0, "get after set");
        CHECK(got != -12345, "option %d read back", k);
        ++accepted;
      } else {
        int got = -12345;
        gm2_get_option(k, &got);
        CHECK(got == before, "a rejected set of option %d changed it (%d -> %d)", k, before, got);
        ++rejected;
      }
    }
  std::printf("option values accepted %d, rejected %d\n", accepted, rejected);
  for (int bad : {0, -1, 23, 1000}) {
    int v = 0;
    expect_error(gm2_set_option(bad, 1), "unknown option", "set unknown key");
    expect_error(gm2_get_option(bad, &v), "unknown option", "get unknown key");
  }
  for (size_t i = 0; i < saved.size(); ++i) gm2_set_option(kKeys[i], saved[i]);
  // per-workspace entry points on a workspace libgm2 never initialised
  char host_buf[64];
  void* ws = host_buf;
  int v = 0;
  expect_error(gm2_workspace_set_option(ws, GM2_OPT_GRID_CAP, 1), "not initialised", "ws set");
  expect_error(gm2_workspace_get_option(ws, GM2_OPT_GRID_CAP, &v), "not initialised", "ws get");
  expect_error(gm2_wait_grad_bucket(ws, 0, nullptr), "not initialised", "wait bucket");
  expect_error(gm2_workspace_join(ws, nullptr), "not initialised", "join");
  expect_error(gm2_workspace_set_collective(ws, nullptr, nullptr), "not initialised", "collective");
  int64_t stat = 0;
  expect_error(gm2_workspace_stat(ws, GM2_STAT_SPLIT_DECODES, &stat), "not initialised", "stat");
  CHECK(gm2_workspace_release(ws) == 0, "release of unknown state is a no-op");
}

// entry points that reach the device: with no GPU (or with arguments refused before any device
// work) each returns an error and leaves nothing behind
static void error_paths() {
  gm2_dims d{300, 128, 8, 64};
  size_t bytes = 0;
  gm2_workspace_size(&d, GM2_BF16, &bytes);
  std::vector<char> host(1 << 16);
  int rc = gm2_workspace_init(&d, GM2_BF16, host.data(), 16, nullptr);  // far too small
  CHECK(rc != 0, "init with a too-small workspace accepted");
  rc = gm2_workspace_init(&d, GM2_BF16, nullptr, bytes, nullptr);
  CHECK(rc != 0, "init with a null workspace accepted");
  rc = gm2_workspace_init(nullptr, GM2_BF16, host.data(), bytes, nullptr);
  CHECK(rc != 0, "init with null dims accepted");
  gm2_batch b{};
  float f = 0.f;
  double loss[GM2_LOSS_SLOTS] = {};
  CHECK(gm2_train_fwd_bwd(&d, GM2_BF16, nullptr, &f, &f, &f, &f, loss, host.data(), nullptr) != 0, "null batch");
  CHECK(gm2_train_fwd_bwd(&d, GM2_BF16, &b, &f, &f, &f, &f, loss, host.data(), nullptr) != 0, "empty batch");
  CHECK(gm2_eval_forward(&d, GM2_BF16, &b, &f, &f, &f, loss, host.data(), nullptr) != 0, "eval empty batch");
  CHECK(gm2_grad_norm(nullptr, GM2_BF16, &f, &f, &f, loss, host.data(), nullptr) != 0, "grad_norm null dims");
  CHECK(gm2_adam_step(nullptr, GM2_BF16, &f, &f, &f, &f, &f, host.data(), nullptr) != 0, "adam null dims");
  CHECK(gm2_sync_shadows(&d, 5, &f, host.data(), nullptr) != 0, "sync_shadows bad precision");
  int64_t ld = 0, ldb = 0, rows = 0;
  size_t nb = 0, nbb = 0;
  CHECK(gm2_resident_layout(-1, 10, GM2_BF16, &ld, &ldb, &rows, &nb, &nbb) != 0, "negative S");
  CHECK(gm2_resident_layout(10, 0, GM2_BF16, &ld, &ldb, &rows, &nb, &nbb) != 0, "zero G");
  CHECK(gm2_reparameterize(-1, &f, &f, &f, &f, nullptr, nullptr, nullptr, nullptr) != 0, "negative n");
  std::string last = gm2_last_error();
  CHECK(!last.empty(), "an error message is kept");
  unsigned flags = 1;
  CHECK(gm2_debug_flags(nullptr) != 0, "debug flags null");
  (void)flags;
}

int main() {
  CHECK(gm2_abi_version() == GM2_ABI_VERSION, "abi version");
  dims_and_layouts();
  options();
  error_paths();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("host_asan: all checks passed\n");
  return 0;
}
