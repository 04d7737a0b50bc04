// Shared device helpers for libgm2 (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gm2 {

typedef uint16_t bf16_t;  // bf16 storage type (bit pattern)
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int kWave = 64;
constexpr int kTile = 128;   // GEMM block tile (M and N); every operand's row count is padded to it
constexpr int kKPad = 64;    // K padding of every operand (covers bf16 BK=64 and f32 BK=32)

__host__ __device__ inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32 (RNE, NaN preserved) on gfx950
  return __builtin_bit_cast(bf16_t, b);
}

// two floats -> packed bf16 pair (lo = a) in one v_cvt_pk_bf16_f32
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
__device__ __forceinline__ uint32_t f2bf2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{a, b}, bf16x2_t));
}

// element-type adaptors: T is float (exact fp32 path) or bf16_t (bf16 MFMA path)
template <typename T> struct E;
template <> struct E<float> {
  static constexpr int KT = 32;  // K elements per 128-byte LDS row chunk
  __device__ static __forceinline__ float ld(const float* p) { return *p; }
  __device__ static __forceinline__ float cvt(float v) { return v; }
};
template <> struct E<bf16_t> {
  static constexpr int KT = 64;
  __device__ static __forceinline__ float ld(const bf16_t* p) { return bf2f(*p); }
  __device__ static __forceinline__ bf16_t cvt(float v) { return f2bf(v); }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// sigmoid_fp32(l) > 0.5  <=>  l > 0x33C00000 (pinned against the reference in tests/golden)
constexpr float kMaskLogitThreshold = 8.940696716308594e-08f;

// ---- debug build (build_native.py --variant debug: -DGM2_DEBUG -> gm2/libgm2_debug.so) ----
// Device-side bounds checks of the index data the kernels follow (gather rows, zero-copy row
// tables, loss target rows, mask group positions, CSR offsets). A failed check ORs its bit into
// this translation unit's flag word with a vector atomic (no trap: the kernel finishes and the
// results are whatever the bad index produced); gm2_debug_flags() reads and clears every unit's word.
enum DebugBit : unsigned {
  kDbgResidentRows = 1u,   // k_resident_rows: rows[i] outside [0, S)
  kDbgGatherRows = 2u,     // k_gather: a negative row index
  kDbgGemmIdx = 4u,        // GEMM zero-copy row table: entry outside [0, idx_lim)
  kDbgMaskPos = 8u,        // k_count_groups: group offsets not ascending / position outside the row
  kDbgCompact = 16u,       // k_compact: an index written outside [off[row], off[row + 1])
  kDbgReconRows = 32u,     // loss epilogue: target-bit row outside [0, idx_lim)
  kDbgTile = 64u,          // a GEMM tile origin outside the padded operand extents
  kDbgBandBlock = 128u,    // band-list overflow: a flagged 256 x 256 block outside the block grid
};
#ifdef GM2_DEBUG
namespace {
__device__ unsigned int g_dbg_flags;  // one per translation unit
}
#define GM2_DBG(cond, bit)                                                                           \
  do {                                                                                              \
    if (!(cond)) __hip_atomic_fetch_or(&g_dbg_flags, (unsigned)(bit), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); \
  } while (0)
// host: this unit's flags, cleared (defines `unsigned fn()`)
#define GM2_DBG_TAKE_FN(fn)                                                                          \
  unsigned fn() {                                                                                   \
    unsigned v = 0, z = 0;                                                                          \
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_dbg_flags), sizeof v) != hipSuccess) return 0x80000000u; \
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_flags), &z, sizeof z) != hipSuccess) return 0x80000000u;   \
    return v;                                                                                       \
  }
#else
#define GM2_DBG(cond, bit) \
  do {                     \
  } while (0)
#endif

}  // namespace gm2
