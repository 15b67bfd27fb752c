// Fused CPVS kernel (gfx950): fps-selected AVPVS frame -> letterbox pad ->
// 4:2:0->4:2:2 chroma conversion -> uyvy422 or v210 packing, in ONE pass.
//
// Replaces the PC branch of create_cpvs (reference lib/ffmpeg.py:1177-1201):
//   -filter:v 'fps=fps=60[,pad=width=W:height=H:x=(ow-iw)/2:y=(oh-ih)/2]'
//   -c:v rawvideo -pix_fmt uyvy422   (8-bit AVPVS)   or   -c:v v210 (10-bit)
// which ffmpeg runs as vf_pad, then an auto-inserted bicubic swscale
// (yuv420p -> uyvy422 via yuv2packedX, yuv420p10le -> yuv422p10le via
// yuv2planeX_10; yuv422p -> uyvy422 via the unscaled interleave), then the
// v210 encoder.  The result is bit-identical to that chain (oracle:
// po_pad + po_sws_scale + po_v210_pack), but the AVPVS is read once and the
// packed frame written once: algorithmic bytes = AVPVS frame + CPVS frame.
//
// Layout: blockIdx.z = frame, blockIdx.y = output row, one lane per 16-byte
// output chunk (8 px of uyvy422, 6 px of v210).  The padded canvas is
// virtual (black outside the AVPVS rectangle); 4:2:0 chroma rows are filtered
// vertically with the plan's bicubic taps (15-bit intermediates: 8-bit <<7,
// 10-bit <<5, then (sum + round) >> 19 / >> 17).  Chroma rows are re-read by
// the two output rows they feed (and the filter halo) from L2.
#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <vector>

#include "common.hpp"
#include "filters.hpp"

namespace pp {

struct CpvsArgs {
    const uint8_t *src[3];
    int64_t sls[3], sfs[3];
    uint8_t *dst;
    int64_t dls, dfs;
    int w, h, cw, ch;     // AVPVS luma / chroma plane sizes
    int W, H;             // canvas
    int ox, oy;           // pad offset (luma, on the chroma grid)
    int vt;               // chroma vertical taps (1 for 4:2:2 sources)
    const int32_t *vpos;  // [H] first padded-chroma row per output row
    const int16_t *vcoef; // [H * vt]
    int chunks;           // 16-B chunks per output line
};

template <typename T>
__device__ inline int sample(const T *row, int x, int x0, int n, int black) {
    const int i = x - x0;
    return (row && i >= 0 && i < n) ? static_cast<int>(row[i]) : black;
}

// DEPTH 8 -> uyvy422, DEPTH 10 -> v210.  V420: source chroma is 4:2:0.
template <int DEPTH, bool V420>
__global__ __launch_bounds__(256) void cpvs_kernel(const CpvsArgs a) {
    using T = typename std::conditional<DEPTH == 8, uint8_t, uint16_t>::type;
    const int frame = blockIdx.z, y = blockIdx.y;
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= a.chunks) return;
    const int by = 16 << (DEPTH - 8), bc = 128 << (DEPTH - 8);
    const int cox = a.ox >> 1;
    // luma row of the canvas
    const T *yrow = (y >= a.oy && y < a.oy + a.h)
                        ? reinterpret_cast<const T *>(a.src[0] + frame * a.sfs[0] + (int64_t)(y - a.oy) * a.sls[0])
                        : nullptr;
    constexpr int PX = DEPTH == 8 ? 8 : 6;   // pixels per 16-B chunk
    constexpr int CPX = PX / 2;
    const int x0 = q * PX;
    int Y[PX], U[CPX], V[CPX];
#pragma unroll
    for (int e = 0; e < PX; ++e) Y[e] = (x0 + e < a.W) ? sample(yrow, x0 + e, a.ox, a.w, by) : 0;
    if constexpr (!V420) {
        const T *ur = yrow ? reinterpret_cast<const T *>(a.src[1] + frame * a.sfs[1] + (int64_t)(y - a.oy) * a.sls[1]) : nullptr;
        const T *vr = yrow ? reinterpret_cast<const T *>(a.src[2] + frame * a.sfs[2] + (int64_t)(y - a.oy) * a.sls[2]) : nullptr;
#pragma unroll
        for (int e = 0; e < CPX; ++e) {
            U[e] = sample(ur, x0 / 2 + e, cox, a.cw, bc);
            V[e] = sample(vr, x0 / 2 + e, cox, a.cw, bc);
        }
    } else {
        // vertical bicubic 2x on the padded 4:2:0 chroma plane (rows [coy, coy + ch) are real)
        const int coy = a.oy >> 1;
        constexpr int SH = DEPTH == 8 ? 7 : 5;          // hScale: (x * 16384) >> (7 | depth-1)
        constexpr int VS = DEPTH == 8 ? 19 : 17;        // yuv2packedX / yuv2planeX_10
        int au[CPX], av[CPX];
#pragma unroll
        for (int e = 0; e < CPX; ++e) au[e] = av[e] = 0;
        const int p0 = a.vpos[y];
        const int16_t *vc = a.vcoef + (int64_t)y * a.vt;
        for (int k = 0; k < a.vt; ++k) {
            const int r = p0 + k - coy;  // AVPVS chroma row, or outside -> black
            const int c = vc[k];
            const bool in = r >= 0 && r < a.ch;
            const T *ur = in ? reinterpret_cast<const T *>(a.src[1] + frame * a.sfs[1] + (int64_t)r * a.sls[1]) : nullptr;
            const T *vr = in ? reinterpret_cast<const T *>(a.src[2] + frame * a.sfs[2] + (int64_t)r * a.sls[2]) : nullptr;
#pragma unroll
            for (int e = 0; e < CPX; ++e) {
                au[e] += (sample(ur, x0 / 2 + e, cox, a.cw, bc) << SH) * c;
                av[e] += (sample(vr, x0 / 2 + e, cox, a.cw, bc) << SH) * c;
            }
        }
        constexpr int MX = (1 << DEPTH) - 1;
#pragma unroll
        for (int e = 0; e < CPX; ++e) {
            U[e] = min(max((au[e] + (1 << (VS - 1))) >> VS, 0), MX);
            V[e] = min(max((av[e] + (1 << (VS - 1))) >> VS, 0), MX);
        }
    }
    uint4 o;
    if constexpr (DEPTH == 8) {
        uint32_t wv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            wv[i] = (uint32_t)U[i] | ((uint32_t)Y[2 * i] << 8) | ((uint32_t)V[i] << 16) | ((uint32_t)Y[2 * i + 1] << 24);
        o = {wv[0], wv[1], wv[2], wv[3]};
        uint8_t *d = a.dst + frame * a.dfs + (int64_t)y * a.dls + (int64_t)q * 16;
        if (x0 + PX <= a.W) {
            *reinterpret_cast<uint4 *>(d) = o;
        } else {
            const uint8_t *b = reinterpret_cast<const uint8_t *>(wv);
            for (int i = 0; i < 2 * (a.W - x0); ++i) d[i] = b[i];
        }
    } else {
        auto c10 = [](int v) -> uint32_t { return v < 4 ? 4u : (v > 1019 ? 1019u : (uint32_t)v); };
        const int full = a.W / 6;
        o = {0, 0, 0, 0};
        if (q < full) {
            o.x = c10(U[0]) | (c10(Y[0]) << 10) | (c10(V[0]) << 20);
            o.y = c10(Y[1]) | (c10(U[1]) << 10) | (c10(Y[2]) << 20);
            o.z = c10(V[1]) | (c10(Y[3]) << 10) | (c10(U[2]) << 20);
            o.w = c10(Y[4]) | (c10(V[2]) << 10) | (c10(Y[5]) << 20);
        } else if (q == full) {  // v210_enc_10 tail, w % 6 in {2..5}
            const int r = a.W - 6 * full;
            if (r >= 2) {
                o.x = c10(U[0]) | (c10(Y[0]) << 10) | (c10(V[0]) << 20);
                const uint32_t val = c10(Y[1]);
                if (r == 2) o.y = val;
                if (r >= 4) {
                    o.y = val | (c10(U[1]) << 10) | (c10(Y[2]) << 20);
                    o.z = c10(V[1]) | (c10(Y[3]) << 10);
                }
            }
        }
        *reinterpret_cast<uint4 *>(a.dst + frame * a.dfs + (int64_t)y * a.dls + (int64_t)q * 16) = o;
    }
}

}  // namespace pp

using namespace pp;

namespace {

// Bicubic 4:2:0 -> 4:2:2 chroma rows of the CLI's auto-inserted converter
// (sws_init_context with chrSrcH = ceil(H/2), chrDstH = H, centred siting),
// compacted; kept per (H) in the context.
struct VTab {
    int vt = 0;
    void *dev = nullptr;
};
std::map<std::pair<pp_ctx *, int>, VTab> g_vtabs;

int get_vtab(pp_ctx *ctx, int H, VTab **out) {
    auto key = std::make_pair(ctx, H);
    auto it = g_vtabs.find(key);
    if (it != g_vtabs.end()) {
        *out = &it->second;
        return PP_OK;
    }
    const int csh = ceil_rshift(H, 1);
    const int inc = (int)((((int64_t)csh << 16) + (H >> 1)) / H);
    FilterBank fb;
    FilterBank::Compact c;
    std::string err;
    if (fb.build(inc, csh, H, 2, 1 << 12, PP_SWS_BICUBIC, PP_SWS_PARAM_DEFAULT, PP_SWS_PARAM_DEFAULT, local_pos(1),
                 local_pos(0), &err) ||
        fb.compact(csh, 1, &c, &err))
        PP_FAIL(PP_ERR_UNSUPPORTED, "cpvs chroma filter: %s", err.c_str());
    VTab t;
    t.vt = c.taps;
    const size_t pb = ((size_t)H * 4 + 255) & ~size_t(255);
    std::vector<uint8_t> host(pb + c.coef.size() * 2);
    std::memcpy(host.data(), c.pos.data(), (size_t)H * 4);
    std::memcpy(host.data() + pb, c.coef.data(), c.coef.size() * 2);
    PP_HIP(hipMalloc(&t.dev, host.size()));
    PP_HIP(hipMemcpy(t.dev, host.data(), host.size(), hipMemcpyHostToDevice));
    auto res = g_vtabs.emplace(key, t);
    *out = &res.first->second;
    return PP_OK;
}

}  // namespace

extern "C" int pp_cpvs_execute(pp_ctx *ctx, int src_fmt, int w, int h, const pp_frames *src, int W, int H, int x,
                               int y, int out_fmt, const pp_frames *dst, int nframes, void *stream) {
    if (!ctx || !src || !dst || nframes < 0) PP_FAIL(PP_ERR_INVALID, "null argument");
    const FmtInfo fi = fmt_info(src_fmt);
    if (!fi.valid || fi.packed || fi.hsub != 1) PP_FAIL(PP_ERR_INVALID, "cpvs source must be 4:2:0 or 4:2:2 planar");
    if (out_fmt == PP_FMT_UYVY422 ? fi.depth != 8 : out_fmt == PP_FMT_V210 ? fi.depth != 10 : true)
        PP_FAIL(PP_ERR_INVALID, "cpvs: uyvy422 needs an 8-bit AVPVS, v210 a 10-bit one");
    if (W < w || H < h || (out_fmt == PP_FMT_UYVY422 && (W & 1))) PP_FAIL(PP_ERR_INVALID, "bad canvas %dx%d", W, H);
    if (x < 0) x = (W - w) / 2;
    if (y < 0) y = (H - h) / 2;
    x = (x >> fi.hsub) << fi.hsub;
    y = (y >> fi.vsub) << fi.vsub;
    if (x + w > W || y + h > H) PP_FAIL(PP_ERR_INVALID, "input exceeds the canvas");
    const int64_t line = out_fmt == PP_FMT_V210 ? pp_v210_linesize(W) : 2LL * W;
    if (dst->linesize[0] < line || ((uintptr_t)dst->data[0] & 15) || (dst->linesize[0] & 15) ||
        (nframes > 1 && (dst->frame_stride[0] & 15)))
        PP_FAIL(PP_ERR_INVALID, "cpvs destination must be 16-B aligned with linesize >= %lld", (long long)line);
    if (nframes == 0) return PP_OK;
    PP_HIP(hipSetDevice(ctx->device));
    CpvsArgs a{};
    for (int p = 0; p < 3; ++p) {
        a.src[p] = (const uint8_t *)src->data[p];
        a.sls[p] = src->linesize[p];
        a.sfs[p] = src->frame_stride[p];
    }
    a.dst = (uint8_t *)dst->data[0];
    a.dls = dst->linesize[0];
    a.dfs = dst->frame_stride[0];
    a.w = w; a.h = h; a.cw = ceil_rshift(w, 1); a.ch = ceil_rshift(h, fi.vsub);
    a.W = W; a.H = H; a.ox = x; a.oy = y;
    a.chunks = (int)(out_fmt == PP_FMT_V210 ? line / 16 : (W + 7) / 8);
    if (fi.vsub) {
        VTab *t;
        int rc = get_vtab(ctx, H, &t);
        if (rc) return rc;
        a.vt = t->vt;
        a.vpos = static_cast<const int32_t *>(t->dev);
        a.vcoef = reinterpret_cast<const int16_t *>(static_cast<const uint8_t *>(t->dev) + (((size_t)H * 4 + 255) & ~size_t(255)));
    }
    hipStream_t st = static_cast<hipStream_t>(stream);
    dim3 grid((a.chunks + 255) / 256, H, nframes);
    if (fi.depth == 8 && fi.vsub)
        hipLaunchKernelGGL((cpvs_kernel<8, true>), grid, dim3(256), 0, st, a);
    else if (fi.depth == 8)
        hipLaunchKernelGGL((cpvs_kernel<8, false>), grid, dim3(256), 0, st, a);
    else if (fi.vsub)
        hipLaunchKernelGGL((cpvs_kernel<10, true>), grid, dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((cpvs_kernel<10, false>), grid, dim3(256), 0, st, a);
    PP_HIP(hipGetLastError());
    return PP_OK;
}
