// Padding, v210 packing and stall-frame compositing kernels (gfx950).
//
//  pp_pad_execute     vf_pad      lib/ffmpeg.py:1183 (PC CPVS), :1209 (tablet)
//  pp_v210_pack       v210enc     lib/test_config.py:208-215 via lib/ffmpeg.py:1198
//  pp_stall_compose   bufferer    p03_generateAvPvs.py:236-243 (spec PP-STALL-1)
//
// All are pure streaming kernels (HBM-bound, no reuse): one lane owns 16 bytes
// of output, blockIdx.z walks the frames of the batch, so one launch covers a
// whole batch.
#include <algorithm>
#include <cstring>
#include <vector>

#include "common.hpp"

namespace pp {

// ---------------------------------------------------------------------------
// vf_pad: out = black, except the (x, y)-shifted input.  EB = bytes per sample.
template <int EB>
__global__ __launch_bounds__(256) void pad_kernel(const uint8_t *src, int64_t sls, int64_t sfs, int iw, int ih,
                                                  uint8_t *dst, int64_t dls, int64_t dfs, int W, int H, int ox,
                                                  int oy, int black) {
    using T = typename std::conditional<EB == 1, uint8_t, uint16_t>::type;
    constexpr int N = 16 / EB;  // samples per lane
    const int frame = blockIdx.z, y = blockIdx.y;
    const T *srow = (y >= oy && y < oy + ih)
                        ? reinterpret_cast<const T *>(src + frame * sfs + (int64_t)(y - oy) * sls)
                        : nullptr;
    T *drow = reinterpret_cast<T *>(dst + frame * dfs + (int64_t)y * dls);
    for (int x = (blockIdx.x * 256 + threadIdx.x) * N; x < W; x += gridDim.x * 256 * N) {
        T v[N];
#pragma unroll
        for (int e = 0; e < N; ++e) {
            const int sx = x + e - ox;
            v[e] = (srow && sx >= 0 && sx < iw) ? srow[sx] : static_cast<T>(black);
        }
        if (x + N <= W && ((reinterpret_cast<uintptr_t>(drow + x) & 15) == 0)) {
            *reinterpret_cast<uint4 *>(drow + x) = *reinterpret_cast<const uint4 *>(v);
        } else {
#pragma unroll
            for (int e = 0; e < N; ++e)
                if (x + e < W) drow[x + e] = v[e];
        }
    }
}

// ---------------------------------------------------------------------------
// v210: 6 pixels -> 4 LE32 words [U0 Y0 V0][Y1 U1 Y2][V1 Y3 U2][Y4 V2 Y5],
// samples clipped to [4, 1019]; line = ceil(w/48)*48*8/3 bytes, zero padded.
__device__ inline uint32_t v210c(uint32_t v) { return v < 4 ? 4 : (v > 1019 ? 1019 : v); }

__global__ __launch_bounds__(256) void v210_kernel(const uint8_t *Yp, const uint8_t *Up, const uint8_t *Vp,
                                                   int64_t yls, int64_t uls, int64_t vls, int64_t yfs, int64_t ufs,
                                                   int64_t vfs, uint8_t *dst, int64_t dls, int64_t dfs, int w,
                                                   int chunks) {
    const int frame = blockIdx.z, row = blockIdx.y;
    const uint16_t *y = reinterpret_cast<const uint16_t *>(Yp + frame * yfs + (int64_t)row * yls);
    const uint16_t *u = reinterpret_cast<const uint16_t *>(Up + frame * ufs + (int64_t)row * uls);
    const uint16_t *v = reinterpret_cast<const uint16_t *>(Vp + frame * vfs + (int64_t)row * vls);
    uint4 *d = reinterpret_cast<uint4 *>(dst + frame * dfs + (int64_t)row * dls);
    const int full = w / 6;
    for (int q = blockIdx.x * 256 + threadIdx.x; q < chunks; q += gridDim.x * 256) {
        uint4 o = {0, 0, 0, 0};
        if (q < full) {
            const int px = 6 * q, cx = 3 * q;
            o.x = v210c(u[cx]) | (v210c(y[px]) << 10) | (v210c(v[cx]) << 20);
            o.y = v210c(y[px + 1]) | (v210c(u[cx + 1]) << 10) | (v210c(y[px + 2]) << 20);
            o.z = v210c(v[cx + 1]) | (v210c(y[px + 3]) << 10) | (v210c(u[cx + 2]) << 20);
            o.w = v210c(y[px + 4]) | (v210c(v[cx + 2]) << 10) | (v210c(y[px + 5]) << 20);
        } else if (q == full) {
            // v210_enc_10 tail for w % 6 in {2..5}
            const int r = w - 6 * full, px = 6 * full, cx = 3 * full;
            if (r >= 2) {
                o.x = v210c(u[cx]) | (v210c(y[px]) << 10) | (v210c(v[cx]) << 20);
                uint32_t val = v210c(y[px + 1]);
                if (r == 2) o.y = val;
                if (r >= 4) {
                    o.y = val | (v210c(u[cx + 1]) << 10) | (v210c(y[px + 2]) << 20);
                    o.z = v210c(v[cx + 1]) | (v210c(y[px + 3]) << 10);
                }
            }
        }
        d[q] = o;
    }
}

// ---------------------------------------------------------------------------
// PP-STALL-1 compositing.  One output frame per blockIdx.z; the spinner
// region (sw x sh luma at (ox, oy)) is alpha-blended, everything else copied
// (or black).  Spinner frame s: Y[sw*sh] Al[sw*sh] U V Ac[(sw>>hs)*(sh>>vs)] u16.
struct StallArgs {
    const uint8_t *src[3];
    int64_t sls[3], sfs[3];
    uint8_t *dst[3];
    int64_t dls[3], dfs[3];
    int32_t idx[2 * 256]; // per output frame of this launch: src index, spinner index
    const uint16_t *spin; // spinner frames
    int64_t spin_stride;  // elements per spinner frame
    int w, h, hs, vs, depth, sw, sh, ox, oy;
};

template <int EB>
__global__ __launch_bounds__(256) void stall_kernel(const StallArgs a) {
    using T = typename std::conditional<EB == 1, uint8_t, uint16_t>::type;
    constexpr int N = 16 / EB;
    const int frame = blockIdx.z;
    const int p = blockIdx.y >= a.h ? (blockIdx.y - a.h >= (a.h >> a.vs) ? 2 : 1) : 0;
    const int y = p == 0 ? blockIdx.y : (blockIdx.y - a.h - (p == 2 ? (a.h >> a.vs) : 0));
    const int W = p ? (a.w >> a.hs) : a.w;
    const int si = a.idx[2 * frame], sp = a.idx[2 * frame + 1];
    const int black = (p ? 128 : 16) << (a.depth - 8);
    const T *srow = si >= 0 ? reinterpret_cast<const T *>(a.src[p] + si * a.sfs[p] + (int64_t)y * a.sls[p]) : nullptr;
    T *drow = reinterpret_cast<T *>(a.dst[p] + frame * a.dfs[p] + (int64_t)y * a.dls[p]);
    // spinner plane geometry
    const int pw = p ? (a.sw >> a.hs) : a.sw, ph = p ? (a.sh >> a.vs) : a.sh;
    const int px0 = p ? (a.ox >> a.hs) : a.ox, py0 = p ? (a.oy >> a.vs) : a.oy;
    const int64_t ysz = (int64_t)a.sw * a.sh, csz = (int64_t)pw * ph;
    const uint16_t *sbase = a.spin + (int64_t)sp * a.spin_stride;
    // layout per spinner frame: Y, Al (sw*sh each), then U, V, Ac (csz each)
    const uint16_t *S = nullptr, *A = nullptr;
    const bool in_rows = sp >= 0 && y >= py0 && y < py0 + ph;
    if (in_rows) {
        S = p == 0 ? sbase : sbase + 2 * ysz + (p == 2 ? csz : 0);
        A = p == 0 ? sbase + ysz : sbase + 2 * ysz + 2 * csz;
        S += (int64_t)(y - py0) * pw;
        A += (int64_t)(y - py0) * pw;
    }
    for (int x = (blockIdx.x * 256 + threadIdx.x) * N; x < W; x += gridDim.x * 256 * N) {
        T v[N];
        if (srow && x + N <= W && ((reinterpret_cast<uintptr_t>(srow + x) & 15) == 0)) {
            *reinterpret_cast<uint4 *>(v) = *reinterpret_cast<const uint4 *>(srow + x);
        } else {
#pragma unroll
            for (int e = 0; e < N; ++e) v[e] = (srow && x + e < W) ? srow[x + e] : static_cast<T>(black);
        }
        if (in_rows && x + N > px0 && x < px0 + pw) {
#pragma unroll
            for (int e = 0; e < N; ++e) {
                const int sx = x + e - px0;
                if (sx >= 0 && sx < pw) {
                    const int al = A[sx];
                    v[e] = static_cast<T>((static_cast<int>(v[e]) * (255 - al) + static_cast<int>(S[sx]) * al + 127) / 255);
                }
            }
        }
        if (x + N <= W && ((reinterpret_cast<uintptr_t>(drow + x) & 15) == 0)) {
            *reinterpret_cast<uint4 *>(drow + x) = *reinterpret_cast<const uint4 *>(v);
        } else {
#pragma unroll
            for (int e = 0; e < N; ++e)
                if (x + e < W) drow[x + e] = v[e];
        }
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
    hipStream_t st = static_cast<hipStream_t>(stream);
    PP_HIP(hipSetDevice(ctx->device));
    for (int p = 0; p < 3; ++p) {
        const int hs = p ? fi.hsub : 0, vs = p ? fi.vsub : 0;
        const int W = ceil_rshift(dw, hs), H = ceil_rshift(dh, vs);
        const int iw = ceil_rshift(sw, hs), ih = ceil_rshift(sh, vs);
        const int black = (p ? 128 : 16) << (fi.depth - 8);
        const int N = fi.depth > 8 ? 8 : 16;
        dim3 grid(std::max(1, (W + 256 * N - 1) / (256 * N)), H, nframes);
        if (fi.depth > 8)
            hipLaunchKernelGGL(pad_kernel<2>, grid, dim3(256), 0, st, (const uint8_t *)src->data[p], src->linesize[p],
                               src->frame_stride[p], iw, ih, (uint8_t *)dst->data[p], dst->linesize[p],
                               dst->frame_stride[p], W, H, x >> hs, y >> vs, black);
        else
            hipLaunchKernelGGL(pad_kernel<1>, grid, dim3(256), 0, st, (const uint8_t *)src->data[p], src->linesize[p],
                               src->frame_stride[p], iw, ih, (uint8_t *)dst->data[p], dst->linesize[p],
                               dst->frame_stride[p], W, H, x >> hs, y >> vs, black);
    }
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
    if (nframes == 0) return PP_OK;
    PP_HIP(hipSetDevice(ctx->device));
    const int chunks = (int)(stride / 16);
    dim3 grid((chunks + 255) / 256, h, nframes);
    hipLaunchKernelGGL(v210_kernel, grid, dim3(256), 0, static_cast<hipStream_t>(stream),
                       (const uint8_t *)src->data[0], (const uint8_t *)src->data[1], (const uint8_t *)src->data[2],
                       src->linesize[0], src->linesize[1], src->linesize[2], src->frame_stride[0],
                       src->frame_stride[1], src->frame_stride[2], (uint8_t *)dst->data[0], dst->linesize[0],
                       dst->frame_stride[0], w, chunks);
    PP_HIP(hipGetLastError());
    return PP_OK;
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
    for (int p = 0; p < 3; ++p) {
        a.src[p] = (const uint8_t *)src->data[p]; a.sls[p] = src->linesize[p]; a.sfs[p] = src->frame_stride[p];
        a.dst[p] = (uint8_t *)dst->data[p]; a.dls[p] = dst->linesize[p]; a.dfs[p] = dst->frame_stride[p];
    }
    a.spin = static_cast<const uint16_t *>(ctx->spin_buf);
    const int cw = ctx->spin_w >> fi.hsub, ch = ctx->spin_h >> fi.vsub;
    a.spin_stride = 2 * (int64_t)ctx->spin_w * ctx->spin_h + 3 * (int64_t)cw * ch;
    a.w = w; a.h = h; a.hs = fi.hsub; a.vs = fi.vsub; a.depth = fi.depth;
    a.sw = need_spin ? ctx->spin_w : 0; a.sh = need_spin ? ctx->spin_h : 0;
    a.ox = ((w - a.sw) / 2) >> fi.hsub << fi.hsub;
    a.oy = ((h - a.sh) / 2) >> fi.vsub << fi.vsub;
    const int rows = h + 2 * (h >> fi.vsub);
    const int N = fi.depth > 8 ? 8 : 16;
    // frame indices travel in the kernel arguments, 256 output frames per launch
    for (int k0 = 0; k0 < nframes; k0 += 256) {
        const int nk = std::min(256, nframes - k0);
        for (int k = 0; k < nk; ++k) {
            a.idx[2 * k] = src_index[k0 + k];
            a.idx[2 * k + 1] = spinner_index[k0 + k];
        }
        StallArgs b = a;
        for (int p = 0; p < 3; ++p) b.dst[p] += k0 * a.dfs[p];
        dim3 grid(std::max(1, (w + 256 * N - 1) / (256 * N)), rows, nk);
        if (fi.depth > 8)
            hipLaunchKernelGGL(stall_kernel<2>, grid, dim3(256), 0, st, b);
        else
            hipLaunchKernelGGL(stall_kernel<1>, grid, dim3(256), 0, st, b);
    }
    PP_HIP(hipGetLastError());
    return PP_OK;
}
