/* libgm2 debug build (genome-minimizer-2_amd/build_native.py --variant debug -> gm2/libgm2_debug.so,
 * compiled with -DGM2_DEBUG): the release library does NOT export these. The debug build adds
 * device-side bounds checks on the index data the kernels follow and host-side layout checks; it
 * computes the same results as the release build (the checks only read). The ASan host build
 * (--variant asan, tools/asan/host_asan.cpp) links the same GM2_DEBUG sources.
 *
 * Not part of the reference's interface: a maintainer's tool for bounds bugs in the workspace
 * layout, the zero-copy row tables and the mask consumers (race detection /
 * sanitizers). */
#ifndef GM2_DEBUG_H
#define GM2_DEBUG_H
#include "gm2.h"

#ifdef __cplusplus
extern "C" {
#endif

/* bits of gm2_debug_flags (genome-minimizer-2_amd/csrc/gm2_common.hpp DebugBit) */
#define GM2_DBG_RESIDENT_ROWS 1  /* a batch row index outside the resident matrix [0, S) */
#define GM2_DBG_GATHER_ROWS 2    /* a negative gather row index */
#define GM2_DBG_GEMM_IDX 4       /* a zero-copy GEMM row-table entry outside the resident operands */
#define GM2_DBG_MASK_POS 8       /* gm2_mask_count_groups: descending group offsets / position past the row */
#define GM2_DBG_COMPACT 16       /* gm2_mask_compact: an index written outside its row's CSR span */
#define GM2_DBG_RECON_ROWS 32    /* loss epilogue: a target-bit row outside the resident bits */
#define GM2_DBG_TILE 64          /* a GEMM tile or K range outside the padded operand extents */
#define GM2_DBG_BAND_BLOCK 128   /* sampling decode: a band-overflow block (or their count) outside the block grid */

/* OR of the failed checks of every kernel since the last call, then cleared (waits for the device) */
int gm2_debug_flags(unsigned* flags);
/* builds the workspace layout of (d, precision) and checks it: every region 256-B aligned, none
 * overlapping another, all inside the total, every named offset a region start */
int gm2_debug_check_layout(const gm2_dims* d, int precision, int64_t* n_regions, int64_t* total);

#ifdef __cplusplus
}
#endif
#endif
