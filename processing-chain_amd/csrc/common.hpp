// Shared host-side helpers of libpixpath.so: error reporting, pixel-format
// table, the context object.  See include/pixpath.h for the ABI.
#pragma once

#ifndef PIXPATH_HOST_ONLY  // `make sanitize`: the host parsers alone, built by g++ under ASan/UBSan
#include <hip/hip_runtime.h>
#endif

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/pixpath.h"

// Measurement knobs (ablation bits, tuning overrides) exist only in the
// ablation build (`make ablate`, tools/ scripts): there PP_KNOB reads the
// environment and PP_ABLATE(x) passes a kernel's ablation bits through.  The
// product library is built without PIXPATH_ABLATE: it never reads the
// environment, and every ablation branch folds to its product path.
#ifdef PIXPATH_ABLATE
#define PP_KNOB(name) std::getenv(name)
#define PP_ABLATE(bits) (bits)
#else
#define PP_KNOB(name) ((const char *)nullptr)
#define PP_ABLATE(bits) 0
#endif

namespace pp {

void set_error(const char *fmt, ...);

#define PP_FAIL(code, ...)                 \
    do {                                   \
        ::pp::set_error(__VA_ARGS__);      \
        return (code);                     \
    } while (0)

#ifndef PIXPATH_HOST_ONLY
#define PP_HIP(expr)                                                              \
    do {                                                                          \
        hipError_t e_ = (expr);                                                   \
        if (e_ != hipSuccess)                                                     \
            PP_FAIL(PP_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));  \
    } while (0)
#endif

// Planar layout of a format: bit depth, chroma subsampling, plane count.
struct FmtInfo {
    int depth;   // bits per sample
    int hsub;    // log2 horizontal chroma subsampling
    int vsub;    // log2 vertical chroma subsampling
    bool packed; // uyvy422 / v210
    bool valid;
};

inline FmtInfo fmt_info(int f) {
    switch (f) {
    case PP_FMT_YUV420P: return {8, 1, 1, false, true};
    case PP_FMT_YUV422P: return {8, 1, 0, false, true};
    case PP_FMT_YUV444P: return {8, 0, 0, false, true};
    case PP_FMT_YUV420P10LE: return {10, 1, 1, false, true};
    case PP_FMT_YUV422P10LE: return {10, 1, 0, false, true};
    case PP_FMT_YUV444P10LE: return {10, 0, 0, false, true};
    case PP_FMT_UYVY422: return {8, 1, 0, true, true};
    case PP_FMT_V210: return {10, 1, 0, true, true};
    default: return {0, 0, 0, false, false};
    }
}

inline int ceil_rshift(int a, int s) { return -((-a) >> s); }

// FFV1 coder / decoder: slices (active lanes) per 64-lane wave.  The range
// coder of a slice is one serial chain and a 600-frame batch has only
// frames x slices chains; fewer lanes per wave trade issue slots for waves.
// Measured (profiles/r3): the encoder's coder is issue-bound per wave (full
// waves best), the decoder waits on its context-block loads (16 lanes best).
// PIXPATH_FFV1_LPW overrides both (1..64; ablation build only).
inline int ffv1_lanes_per_wave(int dflt) {
    static const int v = [] {
        const char *e = PP_KNOB("PIXPATH_FFV1_LPW");
        const int x = e ? std::atoi(e) : 0;
        return x >= 1 && x <= 64 ? x : 0;
    }();
    return v ? v : dflt;
}

// MI355X dispatches the workgroups of a 1-D grid round-robin over its 8 XCDs
// (block b -> XCD b % 8), each with its own L2.  Remapping hardware block `b`
// to logical work item `xcd_remap(b, n)` gives XCD k the contiguous range
// [k*n/8, (k+1)*n/8) in order, so neighbouring work items (strips of one
// frame, bands of one frame range) share an L2 and their halos are fetched
// from HBM once.  A bijection on [0, n) for any n.
constexpr int kXcds = 8;
#ifndef PIXPATH_HOST_ONLY
__host__ __device__
#endif
inline int xcd_remap(int b, int n) {
    const int per = n / kXcds, rem = n % kXcds;
    const int k = b % kXcds, q = b / kXcds;
    return k < rem ? k * (per + 1) + q : rem * (per + 1) + (k - rem) * per + q;
}

struct Ctx {
    int device = 0;
    int cus = 0;  // compute units (persistent grids)
    // spinner animation (PP-STALL-1), device resident
    int spin_fmt = -1, spin_n = 0, spin_w = 0, spin_h = 0;
    void *spin_buf = nullptr; // [n][Y(w*h) A(w*h) U V Ac (cw*ch each)] uint16
};

} // namespace pp

struct pp_ctx : pp::Ctx {};
