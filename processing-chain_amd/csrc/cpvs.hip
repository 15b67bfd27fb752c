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
// Layout: one workgroup per canvas row (1-D grid over frames x rows,
// XCD-remapped so an XCD walks consecutive rows and the 4:2:0 chroma rows the
// vertical filter shares stay in its L2).  The workgroup stages the AVPVS row
// in LDS with coalesced 16-B loads -- for 4:2:0 sources the bicubic-filtered
// chroma row instead (15-bit intermediates: 8-bit <<7, 10-bit <<5, then
// (sum + round) >> 19 / >> 17), each lane filtering 8 samples from the vt
// source rows -- then every lane assembles 16-B output chunks (8 px of
// uyvy422, 6 px of v210) from LDS and stores them.  The padded canvas is
// virtual: samples outside the AVPVS rectangle are black.
#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <vector>

#include "common.hpp"
#include "filters.hpp"

namespace pp {

typedef int16_t v2i16 __attribute__((ext_vector_type(2)));

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
    int ys, cs;           // LDS row strides (samples, whole 16-B groups)
    int aligned;          // all source rows 16-B aligned (vector staging)
};

constexpr int kCpvsLanes = 64;  // one wave per canvas row (4-wave rows: 2.05 vs 1.64 ms, v210 1080p)
constexpr int kCpvsTaps = 4;    // bicubic 2x chroma: at most 4 rows per output row
constexpr int kStageUnroll = 8; // 16-B staging loads a lane keeps in flight

// DEPTH 8 -> uyvy422, DEPTH 10 -> v210.  V420: source chroma is 4:2:0.
template <int DEPTH, bool V420>
__global__ __launch_bounds__(kCpvsLanes) void cpvs_kernel(const CpvsArgs a) {
    using T = typename std::conditional<DEPTH == 8, uint8_t, uint16_t>::type;
    extern __shared__ uint4 lds_raw[];
    T *ly = reinterpret_cast<T *>(lds_raw);
    T *lu = ly + a.ys, *lv = lu + a.cs;
    const int unit = xcd_remap(blockIdx.x, gridDim.x);
    const int frame = unit / a.H, y = unit - frame * a.H;
    const int lane = threadIdx.x;
    const int by = 16 << (DEPTH - 8), bc = 128 << (DEPTH - 8);
    const int iy = y - a.oy;
    const bool live = iy >= 0 && iy < a.h;
    if (live) {
        // LDS = [Y | U | V] rows, each padded to whole 16-B groups: one index
        // space of 16-B pieces over the planes staged (Y only for 4:2:0, whose
        // chroma is filtered below), every load in flight before the writes
        const uint8_t *row0 = a.src[0] + frame * a.sfs[0] + (int64_t)iy * a.sls[0];
        const uint8_t *row1 = a.src[1] + frame * a.sfs[1] + (int64_t)iy * a.sls[1];
        const uint8_t *row2 = a.src[2] + frame * a.sfs[2] + (int64_t)iy * a.sls[2];
        if (a.aligned) {
            const int ny = a.ys * (int)sizeof(T) / 16, nc = V420 ? 0 : a.cs * (int)sizeof(T) / 16;
            const int total = ny + 2 * nc;
            for (int base = 0; base < total; base += kCpvsLanes * kStageUnroll) {
                uint4 r[kStageUnroll];
#pragma unroll
                for (int u = 0; u < kStageUnroll; ++u) {
                    // lanes past the end load piece 0 again (no branch around the
                    // load, so r stays in registers) and do not write it
                    const int i0 = base + u * kCpvsLanes + lane, i = i0 < total ? i0 : 0;
                    const uint8_t *pb = i < ny ? row0 : (i < ny + nc ? row1 : row2);
                    const int j = i < ny ? i : (i < ny + nc ? i - ny : i - ny - nc);
                    r[u] = reinterpret_cast<const uint4 *>(pb)[j];
                }
#pragma unroll
                for (int u = 0; u < kStageUnroll; ++u) {
                    const int i = base + u * kCpvsLanes + lane;
                    if (i < total) lds_raw[i] = r[u];
                }
            }
        } else {
            for (int i = lane; i < a.w; i += kCpvsLanes) ly[i] = reinterpret_cast<const T *>(row0)[i];
            if constexpr (!V420) {
                for (int i = lane; i < a.cw; i += kCpvsLanes) {
                    lu[i] = reinterpret_cast<const T *>(row1)[i];
                    lv[i] = reinterpret_cast<const T *>(row2)[i];
                }
            }
        }
    }
    if constexpr (V420) {
        // vertical bicubic 2x on the padded 4:2:0 chroma plane (rows [coy, coy + ch) are real),
        // 8 samples a lane, the tap rows' loads all in flight
        const int coy = a.oy >> 1;
        constexpr int SH = DEPTH == 8 ? 7 : 5;    // hScale: (x * 16384) >> (7 | depth-1)
        constexpr int VS = DEPTH == 8 ? 19 : 17;  // yuv2packedX / yuv2planeX_10
        constexpr int MX = (1 << DEPTH) - 1;
        const int p0 = a.vpos[y];
        const int16_t *vc = a.vcoef + (int64_t)y * a.vt;
        int coef[kCpvsTaps];
        const uint8_t *ur[kCpvsTaps], *vr[kCpvsTaps];
#pragma unroll
        for (int k = 0; k < kCpvsTaps; ++k) {
            const int r = p0 + k - coy;  // AVPVS chroma row, or outside -> black
            const bool in = k < a.vt && r >= 0 && r < a.ch;
            coef[k] = k < a.vt ? vc[k] : 0;
            ur[k] = in ? a.src[1] + frame * a.sfs[1] + (int64_t)r * a.sls[1] : nullptr;
            vr[k] = in ? a.src[2] + frame * a.sfs[2] + (int64_t)r * a.sls[2] : nullptr;
        }
        // sum_k (x_k << SH) c_k, rounded >> VS  ==  (sum_k x_k c_k + 2^(RS-1)) >> RS:
        // two v_dot2 per sample on (row k, row k+1) sample pairs built by v_perm
        constexpr int RS = VS - SH;
        constexpr int D = sizeof(T) == 2 ? 4 : 2;  // dwords per 8-sample group
        const uint32_t blackw = sizeof(T) == 2 ? (uint32_t)bc * 0x00010001u : (uint32_t)bc * 0x01010101u;
        const v2i16 c01 = {static_cast<int16_t>(coef[0]), static_cast<int16_t>(coef[1])};
        const v2i16 c23 = {static_cast<int16_t>(coef[2]), static_cast<int16_t>(coef[3])};
        const int ngroups = (a.cw + 7) / 8;
        const int nfull = a.aligned ? (a.cs / 8) : 0;  // groups inside the 16-B padded row
        for (int g = lane; g < ngroups; g += kCpvsLanes) {
            uint32_t wu[kCpvsTaps][D], wv[kCpvsTaps][D];
#pragma unroll
            for (int k = 0; k < kCpvsTaps; ++k) {
                if (ur[k] && g < nfull) {
                    if constexpr (D == 4) {
                        const uint4 qu = reinterpret_cast<const uint4 *>(ur[k])[g];
                        const uint4 qv = reinterpret_cast<const uint4 *>(vr[k])[g];
                        wu[k][0] = qu.x; wu[k][1] = qu.y; wu[k][2] = qu.z; wu[k][3] = qu.w;
                        wv[k][0] = qv.x; wv[k][1] = qv.y; wv[k][2] = qv.z; wv[k][3] = qv.w;
                    } else {
                        const uint2 qu = reinterpret_cast<const uint2 *>(ur[k])[g];
                        const uint2 qv = reinterpret_cast<const uint2 *>(vr[k])[g];
                        wu[k][0] = qu.x; wu[k][1] = qu.y;
                        wv[k][0] = qv.x; wv[k][1] = qv.y;
                    }
                } else if (ur[k]) {  // ragged tail or unaligned rows: sample by sample
#pragma unroll
                    for (int d = 0; d < D; ++d) wu[k][d] = wv[k][d] = 0;
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const int x = min(g * 8 + e, a.cw - 1);
                        constexpr int PER = 4 / (int)sizeof(T);
                        const int sh = 8 * (int)sizeof(T) * (e % PER);
                        wu[k][e / PER] |= (uint32_t)reinterpret_cast<const T *>(ur[k])[x] << sh;
                        wv[k][e / PER] |= (uint32_t)reinterpret_cast<const T *>(vr[k])[x] << sh;
                    }
                } else {
#pragma unroll
                    for (int d = 0; d < D; ++d) wu[k][d] = wv[k][d] = blackw;
                }
            }
            uint32_t ou[D], ov[D];
#pragma unroll
            for (int d = 0; d < D; ++d) ou[d] = ov[d] = 0;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                constexpr int PER = 4 / (int)sizeof(T);
                const int dw = e / PER, lo = (e % PER) * (int)sizeof(T);
                // (row k sample e, row k+1 sample e) as two 16-bit lanes
                const uint32_t sel = sizeof(T) == 2
                                         ? (uint32_t)(lo | ((lo + 1) << 8) | ((lo + 4) << 16) | ((lo + 5) << 24))
                                         : (uint32_t)(lo | (0x0c << 8) | ((lo + 4) << 16) | (0x0c << 24));
                auto filt = [&](const uint32_t (&w)[kCpvsTaps][D]) {
                    const v2i16 p01 = __builtin_bit_cast(v2i16, __builtin_amdgcn_perm(w[1][dw], w[0][dw], sel));
                    const v2i16 p23 = __builtin_bit_cast(v2i16, __builtin_amdgcn_perm(w[3][dw], w[2][dw], sel));
                    const int sum = __builtin_amdgcn_sdot2(p23, c23, __builtin_amdgcn_sdot2(p01, c01, 0, false), false);
                    uint32_t v = (uint32_t)min(max((sum + (1 << (RS - 1))) >> RS, 0), MX);
                    // opaque: otherwise two 8-bit results fold into v_ashr_pk_u8_i32, which
                    // leaves the destination's high half as it was (the pre-shift sum) and
                    // the OR below then picks up those bits (measured: +8 on sample 2)
                    asm volatile("" : "+v"(v));
                    return v;
                };
                ou[dw] |= filt(wu) << (8 * lo);
                ov[dw] |= filt(wv) << (8 * lo);
            }
            // lu / lv are padded to whole 16-B groups: the tail lanes write inside them
            if constexpr (D == 4) {
                reinterpret_cast<uint4 *>(lu)[g] = uint4{ou[0], ou[1], ou[2], ou[3]};
                reinterpret_cast<uint4 *>(lv)[g] = uint4{ov[0], ov[1], ov[2], ov[3]};
            } else {
                reinterpret_cast<uint2 *>(lu)[g] = uint2{ou[0], ou[1]};
                reinterpret_cast<uint2 *>(lv)[g] = uint2{ov[0], ov[1]};
            }
        }
    }
    __syncthreads();
    const int cox = a.ox >> 1;
    constexpr int PX = DEPTH == 8 ? 8 : 6;  // pixels per 16-B chunk
    constexpr int CPX = PX / 2;
    uint8_t *drow = a.dst + frame * a.dfs + (int64_t)y * a.dls;
    const bool chroma_live = V420 || live;
    // 8-bit: a chunk wholly inside the AVPVS with the pad offset on an 8-px
    // grid reads its 8 Y and 4 + 4 chroma samples as 3 LDS words and
    // interleaves them with v_perm
    const bool fast8 = DEPTH == 8 && (a.ox & 7) == 0;
    for (int q = lane; q < a.chunks; q += kCpvsLanes) {
        const int x0 = q * PX;
        if constexpr (DEPTH == 8) {
            const int sx0 = x0 - a.ox, csx0 = x0 / 2 - cox;
            if (fast8 && live && sx0 >= 0 && sx0 + 8 <= a.w && csx0 + 4 <= a.cw && x0 + 8 <= a.W) {
                const uint2 yy = *reinterpret_cast<const uint2 *>(ly + sx0);
                const uint32_t uu = *reinterpret_cast<const uint32_t *>(lu + csx0);
                const uint32_t vv = *reinterpret_cast<const uint32_t *>(lv + csx0);
                const uint32_t uv0 = __builtin_amdgcn_perm(vv, uu, 0x05010400u);  // U0 V0 U1 V1
                const uint32_t uv1 = __builtin_amdgcn_perm(vv, uu, 0x07030602u);  // U2 V2 U3 V3
                *reinterpret_cast<uint4 *>(drow + (int64_t)q * 16) =
                    uint4{__builtin_amdgcn_perm(yy.x, uv0, 0x05010400u), __builtin_amdgcn_perm(yy.x, uv0, 0x07030602u),
                          __builtin_amdgcn_perm(yy.y, uv1, 0x05010400u), __builtin_amdgcn_perm(yy.y, uv1, 0x07030602u)};
                continue;
            }
        }
        int Y[PX], U[CPX], V[CPX];
#pragma unroll
        for (int e = 0; e < PX; ++e) {
            const int sx = x0 + e - a.ox;
            Y[e] = (x0 + e >= a.W) ? 0 : (live && sx >= 0 && sx < a.w) ? static_cast<int>(ly[sx]) : by;
        }
#pragma unroll
        for (int e = 0; e < CPX; ++e) {
            const int sx = x0 / 2 + e - cox;
            const bool in = chroma_live && sx >= 0 && sx < a.cw;
            U[e] = in ? static_cast<int>(lu[sx]) : bc;
            V[e] = in ? static_cast<int>(lv[sx]) : bc;
        }
        if constexpr (DEPTH == 8) {
            uint32_t wv[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                wv[i] = (uint32_t)U[i] | ((uint32_t)Y[2 * i] << 8) | ((uint32_t)V[i] << 16) | ((uint32_t)Y[2 * i + 1] << 24);
            uint8_t *d = drow + (int64_t)q * 16;
            if (x0 + PX <= a.W) {
                *reinterpret_cast<uint4 *>(d) = uint4{wv[0], wv[1], wv[2], wv[3]};
            } else {
                for (int i = 0; i < 2 * (a.W - x0); ++i) {  // selects, not a private array
                    const uint32_t w4 = i < 4 ? wv[0] : (i < 8 ? wv[1] : (i < 12 ? wv[2] : wv[3]));
                    d[i] = static_cast<uint8_t>(w4 >> (8 * (i & 3)));
                }
            }
        } else {
            auto c10 = [](int v) -> uint32_t { return v < 4 ? 4u : (v > 1019 ? 1019u : (uint32_t)v); };
            const int full = a.W / 6;
            uint4 o = {0, 0, 0, 0};
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
            *reinterpret_cast<uint4 *>(drow + (int64_t)q * 16) = o;
        }
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
        if (a.vt > kCpvsTaps) PP_FAIL(PP_ERR_UNSUPPORTED, "cpvs chroma filter of %d taps", a.vt);
        a.vpos = static_cast<const int32_t *>(t->dev);
        a.vcoef = reinterpret_cast<const int16_t *>(static_cast<const uint8_t *>(t->dev) + (((size_t)H * 4 + 255) & ~size_t(255)));
    }
    const int es = fi.depth > 8 ? 2 : 1;
    a.ys = (int)(((int64_t)w * es + 15) / 16 * 16 / es);
    a.cs = (int)(((int64_t)a.cw * es + 15) / 16 * 16 / es);
    a.aligned = 1;
    for (int p = 0; p < 3; ++p)
        if (((uintptr_t)src->data[p] & 15) || (src->linesize[p] & 15) || (nframes > 1 && (src->frame_stride[p] & 15)))
            a.aligned = 0;
    const size_t lds = (size_t)(a.ys + 2 * a.cs) * es;
    if (lds > 64 * 1024) PP_FAIL(PP_ERR_UNSUPPORTED, "cpvs: AVPVS width %d exceeds the LDS row stage", w);
    if ((int64_t)H * nframes >= (int64_t)1 << 31) PP_FAIL(PP_ERR_UNSUPPORTED, "cpvs: too many rows in one call");
    hipStream_t st = static_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)(H * nframes));
    if (fi.depth == 8 && fi.vsub)
        hipLaunchKernelGGL((cpvs_kernel<8, true>), grid, dim3(kCpvsLanes), lds, st, a);
    else if (fi.depth == 8)
        hipLaunchKernelGGL((cpvs_kernel<8, false>), grid, dim3(kCpvsLanes), lds, st, a);
    else if (fi.vsub)
        hipLaunchKernelGGL((cpvs_kernel<10, true>), grid, dim3(kCpvsLanes), lds, st, a);
    else
        hipLaunchKernelGGL((cpvs_kernel<10, false>), grid, dim3(kCpvsLanes), lds, st, a);
    PP_HIP(hipGetLastError());
    return PP_OK;
}
