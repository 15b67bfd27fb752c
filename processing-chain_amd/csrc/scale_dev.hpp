// Device-side pieces shared by the scaler kernels (scale.hip: general
// scale_kernel, strip_u16.hip / strip_u8.hip: strip_kernel instances): plane
// jobs, launch arguments, ordered-dither matrix, 16-B buffer loads, v_dot2
// helpers and LDS staging stores.  See scale.hip for the reference semantics.
#pragma once
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "common.hpp"
#include "device.hpp"

namespace pp {

constexpr int kTileW = 256;      // widest output tile (columns); narrower for large downscales
constexpr int kThreads = 256;    // 4 waves
constexpr int kLdsBudget = 40 * 1024;
#ifndef PIXPATH_CHO_MAX
#define PIXPATH_CHO_MAX 32
#endif
#ifndef PIXPATH_SEG_ROWS
#define PIXPATH_SEG_ROWS 540
#endif
constexpr int kChoMax = PIXPATH_CHO_MAX;    // output rows per chunk (upper bound)
constexpr int kSegRows = PIXPATH_SEG_ROWS;  // output rows per segment (target; profiles/r2: 540 beats 256 by ~1.5 %)

static __constant__ uint8_t c_dither[8][8] = {
    {36, 68, 60, 92, 34, 66, 58, 90},  {100, 4, 124, 28, 98, 2, 122, 26},
    {52, 84, 44, 76, 50, 82, 42, 74},  {116, 20, 108, 12, 114, 18, 106, 10},
    {32, 64, 56, 88, 38, 70, 62, 94},  {96, 0, 120, 24, 102, 6, 126, 30},
    {48, 80, 40, 72, 54, 86, 46, 78},  {112, 16, 104, 8, 118, 22, 110, 14},
};

// the same matrix, one row per 64-bit word (byte k = column k): a wave-uniform
// row index makes it one scalar load, the lane's 4 columns one rotate
constexpr uint64_t dither_row64(const uint8_t (&r)[8]) {
    uint64_t v = 0;
    for (int k = 7; k >= 0; --k) v = (v << 8) | r[k];
    return v;
}
constexpr uint8_t kDither[8][8] = {
    {36, 68, 60, 92, 34, 66, 58, 90},  {100, 4, 124, 28, 98, 2, 122, 26},
    {52, 84, 44, 76, 50, 82, 42, 74},  {116, 20, 108, 12, 114, 18, 106, 10},
    {32, 64, 56, 88, 38, 70, 62, 94},  {96, 0, 120, 24, 102, 6, 126, 30},
    {48, 80, 40, 72, 54, 86, 46, 78},  {112, 16, 104, 8, 118, 22, 110, 14},
};
static __constant__ uint64_t c_dither64[8] = {
    dither_row64(kDither[0]), dither_row64(kDither[1]), dither_row64(kDither[2]), dither_row64(kDither[3]),
    dither_row64(kDither[4]), dither_row64(kDither[5]), dither_row64(kDither[6]), dither_row64(kDither[7]),
};

struct PlaneJob {
    int sw, sh, dw, dh;
    int tiles_x, tiles_y, tile_base;  // strips x vertical segments, first block index
    int tw, twl, seg_h, cho; // strip width (= 1 << twl), output rows per segment, output rows per chunk
    int vtp, ring, maxnew, S; // V tap pairs, window rows (even), staged rows per chunk, staged cols
    int dither_off;       // 0 (Y, U) or 3 (V)
    const int32_t *hpos;  // [dw]   window start (absolute source column)
    const int16_t *hcoef; // [dw * HT]
    const int32_t *vbase; // [dh]   first ring row of the window, rounded down to even
    const int32_t *vcoef2; // [dh * vtp] tap pairs (rows base+2j, base+2j+1) packed lo|hi
    const int32_t *tile_c0, *tile_cn; // [tiles_x] staged column window per strip
    const int32_t *chunk_lo, *chunk_hi; // [ceil(dh/cho)] source rows needed by each chunk
    // strip_kernel only
    const int32_t *hbase4;  // [tiles_x * 64] 8-B aligned window base (staged-row sample) per 4-column lane
    const int32_t *hcoefw;  // [tiles_x * 64][4][HW] taps re-laid over the lane's HW dwords (int16 pairs)
    const int32_t *vrow16;  // [dh][16] per output row: window base row (even), then 8 tap pairs (zero padded)
    // chain plans (strip_kernel FUSE != 0, see strip.hpp)
    int fuse;               // 0 as is, 1 identity second stage, 2 second-stage vertical filter through ring2
    int vtp2;               // second-stage V tap pairs (fuse 2)
    int r2mask;             // fuse 2: rows of the circular byte ring2 - 1 (a power of two)
    const int32_t *vrow2;   // [dh2][16] second-stage row records (base row, tap pairs)
    const int32_t *chunk2;  // [nch][4] per chunk: second-stage rows [lo2, hi2), ring2 base row, kept pairs
    const int32_t *seg2;    // fuse 2: [tiles_y][4] per segment: first-stage rows [y0, y1) (chunk aligned,
                            // overlapping by the second stage's halo), second-stage rows [r0, r1) it stores
    int pk_off, pk_step;    // strip_kernel FUSE == 1: byte offset / step of this plane in the uyvy422 row
};

struct ScaleArgs {
    PlaneJob pl[3];
    const uint8_t *src[3];
    int64_t sls[3], sfs[3];
    uint8_t *dst[3];
    int64_t dls[3], dfs[3];
    int nplanes;
    int tiles;    // workgroups per frame (all planes)
    int hshift;   // 7 for 8-bit sources, depth-1 otherwise
    int dither;   // ordered dither (>8-bit source narrowed to 8 bit)
    int vec_src;  // all source rows 16-B aligned
    int vec_dst;  // all destination rows 8-B aligned (4 outputs per lane)
    int debug;    // ablation (measurement only, PIXPATH_SCALE_DEBUG): 1 no V stores, 2 no staging loads, 4 no H pass
};

// Register prefetch of up to kPF 16-byte source chunks per lane (software
// pipelining of the staging: issued before the vertical pass of the previous
// chunk, committed to LDS after it).
constexpr int kPF = 4;

template <typename ST>
struct Prefetch {
    uint4 v[kPF];
};

// Unaligned-source fallback: element loads, zero past the plane edge.
template <typename ST>
__device__ inline uint4 load16_scalar(const ST *g, int col, int sw) {
    constexpr int CH = 16 / sizeof(ST);
    uint4 r = {0, 0, 0, 0};
    ST tmp[CH];
#pragma unroll
    for (int e = 0; e < CH; ++e) tmp[e] = (col + e < sw) ? g[col + e] : ST(0);
    __builtin_memcpy(&r, tmp, 16);
    return r;
}

// Bounds-checked 16-B load through the frame plane's buffer resource: bytes at
// or past num_records read as 0 without touching memory, so lanes with no
// chunk (and the right edge of the plane's last row) need no branch.  Samples
// past a row's end inside the plane come from the next row; the compacted
// filters give them zero weight.
#ifndef PP_SRC_LOAD_AUX
#define PP_SRC_LOAD_AUX 0
#endif
__device__ inline uint4 bload16(__amdgpu_buffer_rsrc_t rs, int off) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, PP_SRC_LOAD_AUX);
    uint4 r;
    __builtin_memcpy(&r, &v, 16);
    return r;
}

typedef int16_t v2i16 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// a.lo*b.lo + a.hi*b.hi + c in the VOP3P form (the compiler's v_dot2c form
// needs the accumulator copied into the destination first)
__device__ inline int dot2_acc(v2i16 a, v2i16 b, int c) {
    int r;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// c + a.lo*b.lo + a.hi*b.hi with b a wave-uniform SGPR and the accumulator c
// a separate VGPR (VOP3P form): the compiler's v_dot2c form would first copy c
// into the destination, one v_mov per output
__device__ inline int dot2_sv(v2i16 a, int32_t b_s, int c) {
    int r;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "s"(b_s), "v"(a), "v"(c));
    return r;
}

// a.lo*b.lo + a.hi*b.hi with a zero accumulator as an inline constant (the
// compiler otherwise zeroes a register for the v_dot2c form)
__device__ inline int dot2_first(v2i16 a, v2i16 b) {
    int r;
    asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// 16-bit sources are stored as s ^ 0x8000 (= s - 32768 as int16) so any u16
// sample is an exact signed operand of v_dot2_i32_i16; the H pass adds the
// 32768 * sum(coef) bias back.  8-bit samples are stored as-is (<= 255).
template <typename ST>
__device__ inline void store16(uint16_t *lds_dst, uint4 v) {
    if constexpr (sizeof(ST) == 2) {
        v.x ^= 0x80008000u; v.y ^= 0x80008000u; v.z ^= 0x80008000u; v.w ^= 0x80008000u;
        *reinterpret_cast<uint4 *>(lds_dst) = v;
    } else {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        uint4 lo, hi;
        lo.x = __builtin_amdgcn_perm(0, w[0], 0x0c010c00u);
        lo.y = __builtin_amdgcn_perm(0, w[0], 0x0c030c02u);
        lo.z = __builtin_amdgcn_perm(0, w[1], 0x0c010c00u);
        lo.w = __builtin_amdgcn_perm(0, w[1], 0x0c030c02u);
        hi.x = __builtin_amdgcn_perm(0, w[2], 0x0c010c00u);
        hi.y = __builtin_amdgcn_perm(0, w[2], 0x0c030c02u);
        hi.z = __builtin_amdgcn_perm(0, w[3], 0x0c010c00u);
        hi.w = __builtin_amdgcn_perm(0, w[3], 0x0c030c02u);
        reinterpret_cast<uint4 *>(lds_dst)[0] = lo;
        reinterpret_cast<uint4 *>(lds_dst)[1] = hi;
    }
}

// ---------------------------------------------------------------------------
// strip_kernel: the common-case scaler (every plane in 256-column strips,
// 16-B aligned source rows, <= 8 vertical tap pairs, <= 10-bit samples).
//
// Same strip/segment/chunk walk and LDS layout as scale_kernel, but every
// loop is wave-uniform (wave = row group, lane = 4 adjacent columns), so the
// control flow is scalar branches instead of exec-mask bookkeeping:
//   H pass: one lane computes 4 adjacent output columns of a row PAIR.  The 4
//     windows share one 8-B aligned base in the staged row (hbase4), read as
//     HW dwords with ds_read_b64 (one read serves all 4 outputs); per output
//     the taps are re-laid over those dwords (hcoefw, zero outside its
//     window), so each output is HW v_dot2_i32_i16 with no realignment, and
//     the 8 results go to the window as one ds_write_b128.
//   V pass: a wave owns an output row; its tap pairs come from a padded
//     [dh][8] table through scalar loads (SGPR operands of v_dot2), the
//     window rows through ds_read_b128 (4 columns x 2 rows), one 8-B store.
//   Kept row pairs are read before the chunk's first barrier and written
//     after it, so the move costs no extra barrier.
// The next chunk's source rows are prefetched into registers right after the
// first barrier, so their HBM latency overlaps both passes.
#define kconst __attribute__((address_space(4)))  // constant address space: uniform loads become s_load
template <typename T>
__device__ inline const kconst T *as_kconst(const void *p) {
    return (const kconst T *)(uintptr_t)p;
}
constexpr int kKeepRegs = 2;  // kept pairs per wave carried in registers (4 waves -> 8 pairs)
constexpr int kStripThreads = kThreads;

template <typename ST>
__device__ inline void store_raw16(uint16_t *lds_dst, uint4 v) {
    if constexpr (sizeof(ST) == 2) {
        *reinterpret_cast<uint4 *>(lds_dst) = v;  // <= 10-bit samples are exact int16 operands
    } else {
        store16<ST>(lds_dst, v);                  // 8-bit: widen to 16-bit
    }
}


using KernelFn = void (*)(const ScaleArgs);
// strip_kernel instances (strip_u16.hip, strip_u8.hip): OUTB 8/10, HW window
// dwords, VTM = largest V tap-pair count over the planes; nullptr if not built
// tw: strip width (= threads) 256 or 512
KernelFn pick_strip_u16(int outb, int hw, int vtm, int tw);
KernelFn pick_strip_u8(int outb, int hw, int vtm, int tw);
// chain plans: first stage to 8 bit, second stage into `out2` (8/10) bits
KernelFn pick_strip_chain_u16(int out2, int hw, int vtm);
KernelFn pick_strip_chain_u8(int out2, int hw, int vtm);
KernelFn pick_strip_luma_u16(int hw, int vtm);  // FUSE 9: a chain's luma launch into 10 bits
KernelFn pick_strip_luma_u8(int hw, int vtm);
KernelFn pick_strip_chroma_u16(int hw, int vtm);  // FUSE 11: a chain's chroma launch into 10 bits
KernelFn pick_strip_chroma_u8(int hw, int vtm);
// GENERIC_UYVY plans: 8-bit samples stored straight into the packed uyvy422 row
KernelFn pick_strip_packed_u16(int hw, int vtm);
KernelFn pick_strip_packed_u8(int hw, int vtm);
int strip_vtm_bucket(int vtp);

}  // namespace pp
