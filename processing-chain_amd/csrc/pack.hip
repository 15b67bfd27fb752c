// Padding, v210 packing and stall-frame compositing kernels (gfx950).
//
//  pp_pad_execute     vf_pad      lib/ffmpeg.py:1183 (PC CPVS), :1209 (tablet)
//  pp_v210_pack       v210enc     lib/test_config.py:208-215 via lib/ffmpeg.py:1198
//  pp_stall_compose   bufferer    p03_generateAvPvs.py:236-243 (spec PP-STALL-1)
//
// All are pure streaming kernels (HBM-bound, no reuse).  Layout: one wave per
// output row of one plane (1-D grid over frames x rows of all three planes,
// XCD-remapped), each lane moving up to four 16-B chunks with every load in
// flight before the first store -- full lanes on chroma rows too, and enough
// bytes in flight per CU to cover HBM latency.  v210 packing goes through the
// fused CPVS kernel (cpvs.hip) with a zero pad.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.hpp"

namespace pp {

constexpr int kRowLanes = 64;  // one wave per row
constexpr int kRowUnroll = 4;  // 16-B chunks a lane keeps in flight

// Per-plane geometry of a row kernel launch.
struct RowPlane {
    const uint8_t *src;
    int64_t sls, sfs;
    uint8_t *dst;
    int64_t dls, dfs;
    int W, rows;       // output plane width (samples) and rows
    int iw, ih;        // source plane size
    int ox, oy;        // source offset on the output plane (pad); 0 for stall
    int black;
    int vec;           // source rows 16-B aligned and ox * EB % 16 == 0: vector loads
    int dvec;          // destination rows 16-B aligned: vector stores
};

// 16-B chunk of output samples [x, x + N) of a row: the source row shifted by
// ox, black outside [0, iw) (and for a null row).
template <typename T>
__device__ inline uint4 shifted_chunk(const T *srow, int x, int ox, int iw, int black, bool vec) {
    constexpr int N = 16 / (int)sizeof(T);
    const int sx = x - ox;
    if (srow && vec && sx >= 0 && sx + N <= iw) return *reinterpret_cast<const uint4 *>(srow + sx);
    T v[N];
#pragma unroll
    for (int e = 0; e < N; ++e) v[e] = (srow && sx + e >= 0 && sx + e < iw) ? srow[sx + e] : static_cast<T>(black);
    uint4 r;
    __builtin_memcpy(&r, v, 16);
    return r;
}

template <typename T>
__device__ inline void put_chunk(T *drow, int x, int W, bool dvec, const uint4 &v) {
    constexpr int N = 16 / (int)sizeof(T);
    if (dvec && x + N <= W) {
        *reinterpret_cast<uint4 *>(drow + x) = v;
    } else {
        T e[N];
        __builtin_memcpy(e, &v, 16);
#pragma unroll
        for (int i = 0; i < N; ++i)
            if (x + i < W) drow[x + i] = e[i];
    }
}

// unit -> (frame, plane, row) of a row-kernel grid over frames x (rows of planes 0, 1, 2)
__device__ inline void row_unit(int unit, const RowPlane *pl, int &frame, int &p, int &y) {
    const int rows = pl[0].rows + pl[1].rows + pl[2].rows;
    frame = unit / rows;
    y = unit - frame * rows;
    p = 0;
    if (y >= pl[0].rows) { y -= pl[0].rows; p = 1; }
    if (p == 1 && y >= pl[1].rows) { y -= pl[1].rows; p = 2; }
}

// ---------------------------------------------------------------------------
// vf_pad: out = black, except the (x, y)-shifted input.  EB = bytes per sample.
struct PadArgs {
    RowPlane pl[3];
};

template <int EB>
__global__ __launch_bounds__(kRowLanes) void pad_kernel(const PadArgs a) {
    using T = typename std::conditional<EB == 1, uint8_t, uint16_t>::type;
    constexpr int N = 16 / EB;
    int frame, p, y;
    row_unit(xcd_remap(blockIdx.x, gridDim.x), a.pl, frame, p, y);
    const RowPlane &g = a.pl[p];
    const int iy = y - g.oy;
    const T *srow = (iy >= 0 && iy < g.ih) ? reinterpret_cast<const T *>(g.src + frame * g.sfs + (int64_t)iy * g.sls)
                                           : nullptr;
    T *drow = reinterpret_cast<T *>(g.dst + frame * g.dfs + (int64_t)y * g.dls);
    const int chunks = (g.W + N - 1) / N;
    for (int q0 = threadIdx.x; q0 < chunks; q0 += kRowLanes * kRowUnroll) {
        uint4 v[kRowUnroll];
#pragma unroll
        for (int u = 0; u < kRowUnroll; ++u) {
            const int q = q0 + u * kRowLanes;
            if (q < chunks) v[u] = shifted_chunk<T>(srow, q * N, g.ox, g.iw, g.black, g.vec);
        }
#pragma unroll
        for (int u = 0; u < kRowUnroll; ++u) {
            const int q = q0 + u * kRowLanes;
            if (q < chunks) put_chunk<T>(drow, q * N, g.W, g.dvec, v[u]);
        }
    }
}

// ---------------------------------------------------------------------------
// PP-STALL-1 compositing.  Output frame k of the launch shows source frame
// idx[2k] (black if < 0) with spinner frame idx[2k+1] (none if < 0): the
// spinner region (sw x sh luma at (ox, oy)) is alpha-blended, everything else
// copied.  Spinner frame s: Y[sw*sh] Al[sw*sh] U V Ac[(sw>>hs)*(sh>>vs)] u16.
struct StallArgs {
    RowPlane pl[3];
    int32_t idx[2 * 256];  // per output frame of this launch: src index, spinner index
    const uint16_t *spin;  // spinner frames
    int64_t spin_stride;   // elements per spinner frame
    int hs, vs, sw, sh, ox, oy;
    int nk, G;             // output frames in this launch, frames per tile
};

#ifndef PIXPATH_STALL_G
#define PIXPATH_STALL_G 6
#endif
template <int EB>
__global__ __launch_bounds__(kRowLanes) void stall_kernel(const StallArgs a) {
    using T = typename std::conditional<EB == 1, uint8_t, uint16_t>::type;
    constexpr int N = 16 / EB;
    // a wave owns one row of one plane for a tile of G consecutive output
    // frames: it loads the source row once (again only where the tile's
    // source index changes: a stall run repeats ONE frozen frame) and stores
    // it G times, blending the spinner row of each frame's spinner index in
    // registers.  Units are tile-major with a tile's rows consecutive, so the
    // waves in flight write adjacent rows of the same G frames.  (Round 5 and
    // earlier: one wave per (row, frame) re-reading the row from L2 for each
    // frame -- 3.0 TB/s of writes, wave dispatch rather than HBM the bound.)
    const int rows = a.pl[0].rows + a.pl[1].rows + a.pl[2].rows;
    const int unit = xcd_remap(blockIdx.x, gridDim.x);
    const int tile = unit / rows, r = unit - tile * rows;
    const int f0 = tile * a.G, f1 = min(a.nk, f0 + a.G);
    if (f0 >= a.nk) return;
    int p = 0, y = r;
    if (y >= a.pl[0].rows) { y -= a.pl[0].rows; p = 1; }
    if (p == 1 && y >= a.pl[1].rows) { y -= a.pl[1].rows; p = 2; }
    const RowPlane &g = a.pl[p];
    // spinner plane geometry
    const int pw = p ? (a.sw >> a.hs) : a.sw, ph = p ? (a.sh >> a.vs) : a.sh;
    const int px0 = p ? (a.ox >> a.hs) : a.ox, py0 = p ? (a.oy >> a.vs) : a.oy;
    const int64_t ysz = (int64_t)a.sw * a.sh, csz = (int64_t)pw * ph;
    const bool spin_row = y >= py0 && y < py0 + ph;
    const int chunks = (g.W + N - 1) / N;
    for (int q0 = threadIdx.x; q0 < chunks; q0 += kRowLanes * kRowUnroll) {
        uint4 base[kRowUnroll];
        int cur = -2;  // no source row loaded (-1 is the black frame)
        for (int f = f0; f < f1; ++f) {
            const int si = a.idx[2 * f], sp = a.idx[2 * f + 1];
            if (si != cur) {  // wave-uniform
                cur = si;
                const T *srow = si >= 0 ? reinterpret_cast<const T *>(g.src + si * g.sfs + (int64_t)y * g.sls) : nullptr;
#pragma unroll
                for (int u = 0; u < kRowUnroll; ++u) {
                    const int q = q0 + u * kRowLanes;
                    if (q < chunks) base[u] = shifted_chunk<T>(srow, q * N, 0, g.W, g.black, g.vec);
                }
            }
            T *drow = reinterpret_cast<T *>(g.dst + f * g.dfs + (int64_t)y * g.dls);
            const uint16_t *S = nullptr, *A = nullptr;
            const bool in_rows = sp >= 0 && spin_row;
            if (in_rows) {
                // layout per spinner frame: Y, Al (sw*sh each), then U, V, Ac (csz each)
                const uint16_t *sbase = a.spin + (int64_t)sp * a.spin_stride;
                S = (p == 0 ? sbase : sbase + 2 * ysz + (p == 2 ? csz : 0)) + (int64_t)(y - py0) * pw;
                A = (p == 0 ? sbase + ysz : sbase + 2 * ysz + 2 * csz) + (int64_t)(y - py0) * pw;
            }
#pragma unroll
            for (int u = 0; u < kRowUnroll; ++u) {
                const int q = q0 + u * kRowLanes, x = q * N;
                if (q >= chunks) continue;
                uint4 v = base[u];
                if (in_rows && x + N > px0 && x < px0 + pw) {
                    T e[N];
                    __builtin_memcpy(e, &v, 16);
#pragma unroll
                    for (int i = 0; i < N; ++i) {
                        const int sx = x + i - px0;
                        if (sx >= 0 && sx < pw) {
                            const int al = A[sx];
                            e[i] = static_cast<T>((static_cast<int>(e[i]) * (255 - al) + static_cast<int>(S[sx]) * al + 127) / 255);
                        }
                    }
                    __builtin_memcpy(&v, e, 16);
                }
                put_chunk<T>(drow, x, g.W, g.dvec, v);
            }
        }
    }
}

// row-kernel plane geometry from the C-ABI frame descriptors
inline void row_planes(RowPlane *pl, const FmtInfo &fi, const pp_frames *src, const pp_frames *dst, int nframes,
                       int sw, int sh, int dw, int dh, int x, int y) {
    const int es = fi.depth > 8 ? 2 : 1;
    for (int p = 0; p < 3; ++p) {
        const int hs = p ? fi.hsub : 0, vs = p ? fi.vsub : 0;
        RowPlane &g = pl[p];
        g.src = (const uint8_t *)src->data[p];
        g.sls = src->linesize[p];
        g.sfs = src->frame_stride[p];
        g.dst = (uint8_t *)dst->data[p];
        g.dls = dst->linesize[p];
        g.dfs = dst->frame_stride[p];
        g.W = ceil_rshift(dw, hs);
        g.rows = ceil_rshift(dh, vs);
        g.iw = ceil_rshift(sw, hs);
        g.ih = ceil_rshift(sh, vs);
        g.ox = x >> hs;
        g.oy = y >> vs;
        g.black = (p ? 128 : 16) << (fi.depth - 8);
        g.vec = !((uintptr_t)g.src & 15) && !(g.sls & 15) && (nframes < 2 || !(g.sfs & 15)) && !((g.ox * es) & 15);
        g.dvec = !((uintptr_t)g.dst & 15) && !(g.dls & 15) && (nframes < 2 || !(g.dfs & 15));
    }
}

// ---- host-side spinner conversion (libavutil/colorspace.h CCIR macros) -----
namespace {
constexpr int kSB = 10;
constexpr int kHalf = 1 << (kSB - 1);
inline int fix(double x) { return static_cast<int>(x * (1 << kSB) + 0.5); }
inline int to_y(int r, int g, int b) {
    return (fix(0.29900 * 219.0 / 255.0) * r + fix(0.58700 * 219.0 / 255.0) * g + fix(0.11400 * 219.0 / 255.0) * b +
            (kHalf + (16 << kSB))) >> kSB;
}
inline int to_u(int r, int g, int b, int shift) {
    return ((-fix(0.16874 * 224.0 / 255.0) * r - fix(0.33126 * 224.0 / 255.0) * g + fix(0.50000 * 224.0 / 255.0) * b +
             (kHalf << shift) - 1) >> (kSB + shift)) + 128;
}
inline int to_v(int r, int g, int b, int shift) {
    return ((fix(0.50000 * 224.0 / 255.0) * r - fix(0.41869 * 224.0 / 255.0) * g - fix(0.08131 * 224.0 / 255.0) * b +
             (kHalf << shift) - 1) >> (kSB + shift)) + 128;
}
}  // namespace

}  // namespace pp

using namespace pp;

extern "C" int pp_pad_execute(pp_ctx *ctx, int fmt, int sw, int sh, const pp_frames *src, int dw, int dh, int x,
                              int y, const pp_frames *dst, int nframes, void *stream) {
    if (!ctx || !src || !dst || nframes < 0) PP_FAIL(PP_ERR_INVALID, "null argument");
    const FmtInfo fi = fmt_info(fmt);
    if (!fi.valid || fi.packed) PP_FAIL(PP_ERR_INVALID, "pad needs a planar format");
    if (x < 0) x = (dw - sw) / 2;  // (ow-iw)/2, truncated like the expression's int conversion
    if (y < 0) y = (dh - sh) / 2;
    x = (x >> fi.hsub) << fi.hsub;  // ff_draw_round_to_sub(.., -1, ..)
    y = (y >> fi.vsub) << fi.vsub;
    if (x + sw > dw || y + sh > dh) PP_FAIL(PP_ERR_INVALID, "input %dx%d at (%d,%d) exceeds %dx%d", sw, sh, x, y, dw, dh);
    if (nframes == 0) return PP_OK;
    PP_HIP(hipSetDevice(ctx->device));
    PadArgs a{};
    row_planes(a.pl, fi, src, dst, nframes, sw, sh, dw, dh, x, y);
    const int64_t units = (int64_t)nframes * (a.pl[0].rows + a.pl[1].rows + a.pl[2].rows);
    if (units >= ((int64_t)1 << 31)) PP_FAIL(PP_ERR_UNSUPPORTED, "pad: too many rows in one call");
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (fi.depth > 8)
        hipLaunchKernelGGL(pad_kernel<2>, dim3((unsigned)units), dim3(kRowLanes), 0, st, a);
    else
        hipLaunchKernelGGL(pad_kernel<1>, dim3((unsigned)units), dim3(kRowLanes), 0, st, a);
    PP_HIP(hipGetLastError());
    return PP_OK;
}

extern "C" int64_t pp_v210_linesize(int w) { return (int64_t)((w + 47) / 48) * 48 * 8 / 3; }

extern "C" int pp_v210_pack(pp_ctx *ctx, int w, int h, const pp_frames *src, const pp_frames *dst, int nframes,
                            void *stream) {
    if (!ctx || !src || !dst || w < 1 || h < 1 || nframes < 0) PP_FAIL(PP_ERR_INVALID, "bad argument");
    const int64_t stride = pp_v210_linesize(w);
    if (dst->linesize[0] < stride || (dst->linesize[0] & 15) || ((uintptr_t)dst->data[0] & 15) ||
        (nframes > 1 && (dst->frame_stride[0] & 15)))
        PP_FAIL(PP_ERR_INVALID, "v210 destination must be 16-B aligned with linesize >= %lld", (long long)stride);
    // yuv422p10le -> v210 is the fused CPVS pass with the canvas = the frame
    return pp_cpvs_execute(ctx, PP_FMT_YUV422P10LE, w, h, src, w, h, 0, 0, PP_FMT_V210, dst, nframes, stream);
}

extern "C" int pp_spinner_upload(pp_ctx *ctx, int fmt, const uint8_t *rgba, int n, int sw, int sh) {
    if (!ctx || !rgba || n < 1 || sw < 2 || sh < 2) PP_FAIL(PP_ERR_INVALID, "bad argument");
    const FmtInfo fi = fmt_info(fmt);
    if (!fi.valid || fi.packed) PP_FAIL(PP_ERR_INVALID, "spinner needs a planar AVPVS format");
    if ((sw & ((1 << fi.hsub) - 1)) || (sh & ((1 << fi.vsub) - 1)))
        PP_FAIL(PP_ERR_INVALID, "spinner %dx%d not on the chroma grid", sw, sh);
    const int cw = sw >> fi.hsub, ch = sh >> fi.vsub, shift = fi.hsub + fi.vsub, up = fi.depth - 8;
    const int64_t per = 2 * (int64_t)sw * sh + 3 * (int64_t)cw * ch;
    std::vector<uint16_t> host((size_t)per * n);
    for (int f = 0; f < n; ++f) {
        const uint8_t *img = rgba + (size_t)f * sw * sh * 4;
        uint16_t *Y = host.data() + (size_t)f * per, *Al = Y + sw * sh, *U = Al + sw * sh, *V = U + cw * ch,
                 *Ac = V + cw * ch;
        for (int i = 0; i < sw * sh; ++i) {
            Y[i] = (uint16_t)(to_y(img[4 * i], img[4 * i + 1], img[4 * i + 2]) << up);
            Al[i] = img[4 * i + 3];
        }
        for (int cy = 0; cy < ch; ++cy)
            for (int cx = 0; cx < cw; ++cx) {
                int r = 0, g = 0, b = 0, al = 0;
                for (int dy = 0; dy < (1 << fi.vsub); ++dy)
                    for (int dx = 0; dx < (1 << fi.hsub); ++dx) {
                        const uint8_t *q = img + 4 * ((size_t)((cy << fi.vsub) + dy) * sw + (cx << fi.hsub) + dx);
                        r += q[0]; g += q[1]; b += q[2]; al += q[3];
                    }
                U[cy * cw + cx] = (uint16_t)(to_u(r, g, b, shift) << up);
                V[cy * cw + cx] = (uint16_t)(to_v(r, g, b, shift) << up);
                Ac[cy * cw + cx] = (uint16_t)((al + ((1 << shift) >> 1)) >> shift);
            }
    }
    PP_HIP(hipSetDevice(ctx->device));
    if (ctx->spin_buf) PP_HIP(hipFree(ctx->spin_buf));
    ctx->spin_buf = nullptr;
    PP_HIP(hipMalloc(&ctx->spin_buf, host.size() * 2));
    PP_HIP(hipMemcpy(ctx->spin_buf, host.data(), host.size() * 2, hipMemcpyHostToDevice));
    ctx->spin_fmt = fmt; ctx->spin_n = n; ctx->spin_w = sw; ctx->spin_h = sh;
    return PP_OK;
}

extern "C" int pp_stall_compose(pp_ctx *ctx, int fmt, int w, int h, const pp_frames *src, const int32_t *src_index,
                                const int32_t *spinner_index, const pp_frames *dst, int nframes, void *stream) {
    if (!ctx || !src || !dst || !src_index || !spinner_index || nframes < 0) PP_FAIL(PP_ERR_INVALID, "null argument");
    const FmtInfo fi = fmt_info(fmt);
    if (!fi.valid || fi.packed) PP_FAIL(PP_ERR_INVALID, "stall compose needs a planar format");
    if ((w & ((1 << fi.hsub) - 1)) || (h & ((1 << fi.vsub) - 1))) PP_FAIL(PP_ERR_INVALID, "odd frame size");
    bool need_spin = false;
    for (int k = 0; k < nframes; ++k) need_spin |= spinner_index[k] >= 0;
    if (need_spin && (ctx->spin_fmt != fmt || !ctx->spin_buf))
        PP_FAIL(PP_ERR_INVALID, "no spinner uploaded for format %d", fmt);
    for (int k = 0; k < nframes; ++k)
        if (spinner_index[k] >= ctx->spin_n) PP_FAIL(PP_ERR_INVALID, "spinner index %d out of range", spinner_index[k]);
    if (nframes == 0) return PP_OK;
    hipStream_t st = static_cast<hipStream_t>(stream);
    PP_HIP(hipSetDevice(ctx->device));
    StallArgs a{};
    row_planes(a.pl, fi, src, dst, nframes, w, h, w, h, 0, 0);
    a.spin = static_cast<const uint16_t *>(ctx->spin_buf);
    const int cw = ctx->spin_w >> fi.hsub, ch = ctx->spin_h >> fi.vsub;
    a.spin_stride = 2 * (int64_t)ctx->spin_w * ctx->spin_h + 3 * (int64_t)cw * ch;
    a.hs = fi.hsub; a.vs = fi.vsub;
    a.sw = need_spin ? ctx->spin_w : 0; a.sh = need_spin ? ctx->spin_h : 0;
    a.ox = ((w - a.sw) / 2) >> fi.hsub << fi.hsub;
    a.oy = ((h - a.sh) / 2) >> fi.vsub << fi.vsub;
    const int rows = a.pl[0].rows + a.pl[1].rows + a.pl[2].rows;
    // frame indices travel in the kernel arguments, 256 output frames per launch
    for (int k0 = 0; k0 < nframes; k0 += 256) {
        const int nk = std::min(256, nframes - k0);
        for (int k = 0; k < nk; ++k) {
            a.idx[2 * k] = src_index[k0 + k];
            a.idx[2 * k + 1] = spinner_index[k0 + k];
        }
        StallArgs b = a;
        for (int p = 0; p < 3; ++p) b.pl[p].dst += k0 * a.pl[p].dfs;
        b.nk = nk;
        // frames per wave (one source load, G stores of the row).  Round 2,
        // one wave per (row, frame) in tiles of G: G = 1 1.34 ms, 2
        // 1.09-1.12, 3 1.07-1.10, 4 1.12, 6 1.03-1.05, 8 1.33, 16 1.42, 64 1.55
        // (power-of-two tiles alias the frames' rows onto the same HBM channels)
        b.G = PIXPATH_STALL_G;
        const dim3 grid((unsigned)((nk + b.G - 1) / b.G * rows));
        if (fi.depth > 8)
            hipLaunchKernelGGL(stall_kernel<2>, grid, dim3(kRowLanes), 0, st, b);
        else
            hipLaunchKernelGGL(stall_kernel<1>, grid, dim3(kRowLanes), 0, st, b);
    }
    PP_HIP(hipGetLastError());
    return PP_OK;
}
