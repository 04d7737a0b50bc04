// Tuning options of libgm2 (gm2.h GM2_OPT_*): per-workspace copies, process defaults, and the
// per-call scope through which the launchers read them. Host code only.
#include <cstdio>
#include <cstdlib>
#include <mutex>

#include "../../include/gm2.h"
#include "gm2_kernels.hpp"

namespace gm2 {

namespace {

std::mutex& defaults_mutex() {
  static std::mutex mu;
  return mu;
}

Options& defaults_locked() {
  static Options d = [] {
    Options o;
    const char* pp = std::getenv("GM2_GEMM_PP");
    if (pp && pp[0] == '0') o.gemm_pp = 0;
    const char* side = std::getenv("GM2_SIDE_STREAM");
    if (side && side[0] == '0') o.side_stream = 0;
    // GM2_OPTS="key=value,key=value" (gm2.h GM2_OPT_* numbers): process defaults for same-box A/Bs;
    // a malformed or refused entry is ignored
    if (const char* e = std::getenv("GM2_OPTS")) {
      int key = 0, value = 0, used = 0;
      while (*e && std::sscanf(e, "%d=%d%n", &key, &value, &used) == 2) {
        try {
          option_set(o, key, value);
        } catch (const Gm2Error&) {
        }
        e += used;
        if (*e == ',') ++e;
      }
    }
    return o;
  }();
  return d;
}

thread_local Options tl_opts;
thread_local int tl_active = 0;

}  // namespace

void option_set(Options& o, int key, int value) {
  switch (key) {
    case GM2_OPT_GEMM_PP: o.gemm_pp = value ? 1 : 0; break;
    case GM2_OPT_SIDE_STREAM: o.side_stream = value ? 1 : 0; break;
    case GM2_OPT_RECON_TILE:
      if (value != 0 && value != 128 && value != 256) throw Gm2Error("recon tile %d: 0, 128 or 256", value);
      o.recon_tile = value;
      break;
    case GM2_OPT_SMALL_SPLIT: o.small_split = std::max(1, std::min(value, 8)); break;
    case GM2_OPT_BN_EPILOGUE: o.bn_epilogue = value ? 1 : 0; break;
    case GM2_OPT_SMALL_WAVES:
      if (value != 4 && value != 8) throw Gm2Error("small waves %d: 4 or 8", value);
      o.small_waves = value;
      break;
    case GM2_OPT_GRID_CAP:
      if (value < 0 || value > 7) throw Gm2Error("grid cap bits %d: 0..7", value);
      o.grid_cap = value;
      break;
    case GM2_OPT_INPUT_CHUNKS:
      if (value != 1 && value != 4) throw Gm2Error("input chunks %d: 1 or 4", value);
      o.input_chunks = value;
      break;
    case GM2_OPT_SYNC_BN: o.sync_bn = value ? 1 : 0; break;
    case GM2_OPT_DEFER_OUTPUT_ADAM:
      if (value < 0 || value > 16) throw Gm2Error("deferred output-layer update: %d workgroups per CU (0..16)", value);
      o.defer_adam = value;
      break;
    case GM2_OPT_GRAD_BUCKETS: o.grad_buckets = value ? 1 : 0; break;
    case GM2_OPT_SAMPLE_SPLIT: o.sample_split = value ? 1 : 0; break;
    case GM2_OPT_SAMPLE_SINGLE: o.sample_single = value ? 1 : 0; break;
    case GM2_OPT_SAMPLE_BAND_CAP:
      if (value < 1 || value > (int)kBandShardCap) throw Gm2Error("band list cap %d: 1..%u", value, kBandShardCap);
      o.band_cap = value;
      break;
    case GM2_OPT_SAMPLE_SINGLE_BOUND:
      if (value < 1 || value > 1000000) throw Gm2Error("single-tier bound %d (x 1e-3): 1..1000000", value);
      o.single_bound_milli = value;
      break;
    default: throw Gm2Error("unknown option %d", key);
  }
}

int option_get(const Options& o, int key) {
  switch (key) {
    case GM2_OPT_GEMM_PP: return o.gemm_pp;
    case GM2_OPT_SIDE_STREAM: return o.side_stream;
    case GM2_OPT_RECON_TILE: return o.recon_tile;
    case GM2_OPT_SMALL_SPLIT: return o.small_split;
    case GM2_OPT_BN_EPILOGUE: return o.bn_epilogue;
    case GM2_OPT_SMALL_WAVES: return o.small_waves;
    case GM2_OPT_GRID_CAP: return o.grid_cap;
    case GM2_OPT_INPUT_CHUNKS: return o.input_chunks;
    case GM2_OPT_SYNC_BN: return o.sync_bn;
    case GM2_OPT_DEFER_OUTPUT_ADAM: return o.defer_adam;
    case GM2_OPT_GRAD_BUCKETS: return o.grad_buckets;
    case GM2_OPT_SAMPLE_SPLIT: return o.sample_split;
    case GM2_OPT_SAMPLE_SINGLE: return o.sample_single;
    case GM2_OPT_SAMPLE_BAND_CAP: return o.band_cap;
    case GM2_OPT_SAMPLE_SINGLE_BOUND: return o.single_bound_milli;
    default: throw Gm2Error("unknown option %d", key);
  }
}

Options default_options() {
  std::lock_guard<std::mutex> lk(defaults_mutex());
  return defaults_locked();
}

void set_default_option(int key, int value) {
  std::lock_guard<std::mutex> lk(defaults_mutex());
  Options o = defaults_locked();
  option_set(o, key, value);  // validates before anything changes
  defaults_locked() = o;
}

const Options& opts() {
  if (!tl_active) tl_opts = default_options();  // a launcher reached outside any scope
  return tl_opts;
}

OptionScope::OptionScope(const Options& o) : saved(tl_opts), was(tl_active) {
  tl_opts = o;
  tl_active = 1;
}

OptionScope::~OptionScope() {
  tl_opts = saved;
  tl_active = was;
}

}  // namespace gm2
