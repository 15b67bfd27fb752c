// FFV1 version 3 intra encoder on gfx950: the
// AVPVS intermediate the reference writes with
// `-c:v ffv1 -threads 4 -level 3 -coder 1 -context 1 -slicecrc 1`
// (lib/ffmpeg.py:993, :1047).  Bitstream per RFC 9043 / FFmpeg 7.0 ffv1enc.c;
// the encoder's choices (range coder with the default state table, a 3-input
// 666-context quantisation set, every frame a keyframe, caller-chosen slice
// grid, slice CRCs) are listed in oracle/ffv1_oracle.c and DESIGN.md.
//
// GPU shape: the range coder of a slice is one serial dependency chain (each
// binary decision updates `low/range` and an adaptive state byte), so the
// unit of parallelism is the slice: ONE LANE PER SLICE, every slice of every
// frame of the batch at once (600 frames x 16 slices = 9600 lanes).  A lane
// walks its slice's Y, Cb, Cr samples in raster order: context from
// (L - TL, TL - T, T - TR), median prediction, residual folded to the bit
// depth, then put_symbol's binary decisions through its own context states
// (2 sets x 666 x 32 B in HBM, primed to 128 by a memset; hot contexts stay in
// L1/L2) and the state-transition tables in LDS.  Bytes go to a per-slice
// output region with a running CRC-32 (LDS table); ffv1_pack_kernel then lays
// the slices out as frame packets with their 8-byte footers.
// Latency-bound by construction (dependent state loads), not HBM-bound: the
// figure of merit is frames/s against the CPU restatement (bench --workload ffv1).
#include <algorithm>
#include <cstring>
#include <memory>
#include <vector>

#include "common.hpp"
#include "device.hpp"

namespace pp {

constexpr int kFfv1Ctx = 666;   // (11^3 + 1) / 2 contexts per plane set
constexpr int kCtxSize = 32;    // state bytes per context
constexpr int kStateBytes = 2 * kFfv1Ctx * kCtxSize + 64;  // + slice-header states, keyframe and end bits
constexpr int kSlotStride = 40;  // LDS bytes per lane for the cached context

// ---- host range coder (configuration record) and state tables -------------
struct HostRC {
    int low = 0, range = 0xFF00, oc = 0, ob = -1;
    uint8_t zero[256], one[256];
    std::vector<uint8_t> out;
    void byte(int v) { out.push_back((uint8_t)v); }
    void renorm() {
        while (range < 0x100) {
            if (ob < 0) {
                ob = low >> 8;
            } else if (low <= 0xFF00) {
                byte(ob);
                for (; oc; oc--) byte(0xFF);
                ob = low >> 8;
            } else if (low >= 0x10000) {
                byte(ob + 1);
                for (; oc; oc--) byte(0x00);
                ob = (low >> 8) - 0x100;
            } else {
                oc++;
            }
            low = (low & 0xFF) << 8;
            range <<= 8;
        }
    }
    void rac(uint8_t *st, int bit) {
        const int r1 = (range * *st) >> 8;
        if (!bit) {
            range -= r1;
            *st = zero[*st];
        } else {
            low += range - r1;
            range = r1;
            *st = one[*st];
        }
        renorm();
    }
    void symbol(uint8_t *st, int v) {  // unsigned
        if (!v) {
            rac(st, 1);
            return;
        }
        int e = 0;
        while ((v >> (e + 1)) > 0) ++e;
        rac(st, 0);
        for (int i = 0; i < e; i++) rac(st + 1 + std::min(i, 9), 1);
        rac(st + 1 + std::min(e, 9), 0);
        for (int i = e - 1; i >= 0; i--) rac(st + 22 + std::min(i, 9), (v >> i) & 1);
    }
    size_t terminate() {
        range = 0xFF;
        low += 0xFF;
        renorm();
        range = 0xFF;
        renorm();
        return out.size();
    }
};

// ff_build_rac_states(c, 0.05 * 2^32, 256 - 8): the default state-transition table
void rac_states(uint8_t zero[256], uint8_t one[256]) {
    const int64_t kOne = (int64_t)1 << 32;
    const int64_t factor = (int64_t)(0.05 * (double)((int64_t)1 << 32));
    const int max_p = 256 - 8;
    std::memset(zero, 0, 256);
    std::memset(one, 0, 256);
    int64_t p = kOne / 2;
    int last_p8 = 0;
    for (int i = 0; i < 128; i++) {
        int p8 = (int)((256 * p + kOne / 2) >> 32);
        if (p8 <= last_p8) p8 = last_p8 + 1;
        if (last_p8 && last_p8 < 256 && p8 <= max_p) one[last_p8] = (uint8_t)p8;
        p += ((kOne - p) * factor + kOne / 2) >> 32;
        last_p8 = p8;
    }
    for (int i = 256 - max_p; i <= max_p; i++) {
        if (one[i]) continue;
        p = (i * kOne + 128) >> 8;
        p += ((kOne - p) * factor + kOne / 2) >> 32;
        int p8 = (int)((256 * p + kOne / 2) >> 32);
        if (p8 <= i) p8 = i + 1;
        if (p8 > max_p) p8 = max_p;
        one[i] = (uint8_t)p8;
    }
    for (int i = 1; i < 255; i++) zero[i] = (uint8_t)(256 - one[256 - i]);
}

// AV_CRC_32_IEEE: polynomial 0x04C11DB7, MSB first, initial 0, no final xor
void crc_table(uint32_t t[256]) {
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i << 24;
        for (int j = 0; j < 8; j++) c = (c << 1) ^ ((c & 0x80000000u) ? 0x04C11DB7u : 0u);
        t[i] = c;
    }
}

// quantiser of the context inputs on (d & 0xFF): min(5, bit length of |d|), odd-mirrored
inline int quant_host(int i) {
    if (i >= 128) return -quant_host(i == 128 ? 127 : 256 - i);
    int q = 0;
    while (i) { q++; i >>= 1; }
    return std::min(q, 5);
}

// ---- device ---------------------------------------------------------------
struct Ffv1Args {
    const uint8_t *src[3];
    int64_t ls[3], fs[3];
    int w, h, bytes, bits, hsub, vsub, nh, nv, nslices;  // nslices = frames * nh * nv
    uint8_t *out;           // [nslices][cap]
    int64_t cap;
    uint8_t *states;        // [nslices][kStateBytes], primed to 128
    int64_t *sizes;         // [nslices] coded bytes, -1 = overflow
    uint32_t *crcs;         // [nslices] CRC-32 of the coded bytes
    const uint8_t *tables;  // zero[256], one[256], crc table (1 KB)
};

__device__ inline int dquant(int d) {  // d already & 0xFF
    const int m = d < 128 ? d : (d == 128 ? 127 : 256 - d);
    const int q = min(32 - __clz(m), 5);
    return d < 128 ? q : -q;
}

__device__ inline int median3(int a, int b, int c) {
    return max(min(a, b), min(max(a, b), c));
}

// The slice's range coder (rangecoder.c put_rac / renorm_encoder) and
// put_symbol; every method force-inlined so the coder lives in registers.
struct DevRC {
    int low, range, oc, ob;
    uint8_t *p, *end;
    uint32_t crc;
    bool over;
    const uint8_t *zero, *one;
    const uint32_t *crc_tab;

    __device__ __forceinline__ void emit(int v) {
        if (p < end) {
            *p++ = (uint8_t)v;
            crc = (crc << 8) ^ crc_tab[(crc >> 24) ^ (uint32_t)(v & 0xFF)];
        } else {
            over = true;
        }
    }
    __device__ __forceinline__ void renorm() {
        while (range < 0x100) {
            if (ob < 0) {
                ob = low >> 8;
            } else if (low <= 0xFF00) {
                emit(ob);
                for (; oc; oc--) emit(0xFF);
                ob = low >> 8;
            } else if (low >= 0x10000) {
                emit(ob + 1);
                for (; oc; oc--) emit(0x00);
                ob = (low >> 8) - 0x100;
            } else {
                oc++;
            }
            low = (low & 0xFF) << 8;
            range <<= 8;
        }
    }
    // one binary decision with the adaptive state byte at *st (HBM/L2)
    __device__ __forceinline__ void rac(uint8_t *st, int bit) {
        const int sv = *st;
        const int r1 = (range * sv) >> 8;
        if (!bit) {
            range -= r1;
            *st = zero[sv];
        } else {
            low += range - r1;
            range = r1;
            *st = one[sv];
        }
        renorm();
    }
    __device__ __forceinline__ void symbol(uint8_t *st, int v, bool is_signed) {
        if (!v) {
            rac(st, 1);
            return;
        }
        const int av = v < 0 ? -v : v;
        const int e = 31 - __clz(av);
        rac(st, 0);
        for (int i = 0; i < e; i++) rac(st + 1 + min(i, 9), 1);
        rac(st + 1 + min(e, 9), 0);
        for (int i = e - 1; i >= 0; i--) rac(st + 22 + min(i, 9), (av >> i) & 1);
        if (is_signed) rac(st + 11 + min(e, 10), v < 0);
    }
};

template <typename T>
__device__ inline int ldpx(const uint8_t *row, int x) {
    return reinterpret_cast<const T *>(row)[x];
}

__global__ __launch_bounds__(64) void ffv1_slice_kernel(const Ffv1Args a) {
    __shared__ uint8_t s_zero[256], s_one[256];
    __shared__ uint32_t s_crc[256];
    // the 32 state bytes of the context the lane is coding with, cached in LDS
    // (stride 40 B: 2-way bank conflicts at most); written back to HBM when the
    // lane switches context, so put_symbol's ~10 dependent state accesses per
    // sample are LDS round trips instead of L1/L2 ones
    __shared__ __align__(16) uint8_t s_ctx[64 * kSlotStride];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        s_zero[i] = a.tables[i];
        s_one[i] = a.tables[256 + i];
        s_crc[i] = reinterpret_cast<const uint32_t *>(a.tables + 512)[i];
    }
    __syncthreads();
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= a.nslices) return;
    const int per = a.nh * a.nv;
    const int frame = g / per, s = g - frame * per;
    const int sy = s / a.nh, sx = s - sy * a.nh;
    uint8_t *const st0 = a.states + (int64_t)g * kStateBytes;
    DevRC c;
    c.low = 0; c.range = 0xFF00; c.oc = 0; c.ob = -1;
    c.p = a.out + (int64_t)g * a.cap;
    c.end = c.p + a.cap;
    c.crc = 0;
    c.over = false;
    c.zero = s_zero; c.one = s_one; c.crc_tab = s_crc;
    // header: keyframe bit (first slice of a frame), slice header with its own
    // 32 states -- all in the slice's state block (primed to 128), not in
    // private memory
    uint8_t *const hs = st0 + 2 * kFfv1Ctx * kCtxSize;
    if (s == 0) c.rac(hs + 32, 1);
    // slice x, y, width - 1, height - 1 (slice units), table set of Y and of
    // Cb/Cr, picture_structure 3 (progressive), SAR 1:1 (setsar=1/1)
    for (int i = 0; i < 9; i++) c.symbol(hs, i == 0 ? sx : i == 1 ? sy : i == 6 ? 3 : i >= 7 ? 1 : 0, false);

    const int x0 = (int)((int64_t)sx * a.w / a.nh), x1 = (int)((int64_t)(sx + 1) * a.w / a.nh);
    const int y0 = (int)((int64_t)sy * a.h / a.nv), y1 = (int)((int64_t)(sy + 1) * a.h / a.nv);
    const int mask = (1 << a.bits) - 1, half = 1 << (a.bits - 1);
    uint8_t *const slot = s_ctx + threadIdx.x * kSlotStride;
    int cur_key = -1;  // (plane set, context) held in `slot`
    auto switch_ctx = [&](int key) {
        if (cur_key >= 0) {
            uint2 *g = reinterpret_cast<uint2 *>(st0 + cur_key * kCtxSize);
            const uint2 *l = reinterpret_cast<const uint2 *>(slot);
#pragma unroll
            for (int i = 0; i < 4; i++) g[i] = l[i];
        }
        const uint2 *g = reinterpret_cast<const uint2 *>(st0 + key * kCtxSize);
        uint2 *l = reinterpret_cast<uint2 *>(slot);
        uint2 v[4];
#pragma unroll
        for (int i = 0; i < 4; i++) v[i] = g[i];
#pragma unroll
        for (int i = 0; i < 4; i++) l[i] = v[i];
        cur_key = key;
    };
    for (int p = 0; p < 3; p++) {
        const int pw = p ? ((x1 - x0) + (1 << a.hsub) - 1) >> a.hsub : x1 - x0;
        const int ph = p ? ((y1 - y0) + (1 << a.vsub) - 1) >> a.vsub : y1 - y0;
        const int px0 = p ? x0 >> a.hsub : x0, py0 = p ? y0 >> a.vsub : y0;
        // plane fields by selects, not a runtime index into the argument arrays (private memory)
        const uint8_t *src = p == 0 ? a.src[0] : p == 1 ? a.src[1] : a.src[2];
        const int64_t ls = p == 0 ? a.ls[0] : p == 1 ? a.ls[1] : a.ls[2];
        const int64_t fs = p == 0 ? a.fs[0] : p == 1 ? a.fs[1] : a.fs[2];
        const uint8_t *base = src + frame * fs + (int64_t)py0 * ls + (int64_t)px0 * a.bytes;
        const int key0 = p ? kFfv1Ctx : 0;
        for (int y = 0; y < ph; y++) {
            const uint8_t *row = base + (int64_t)y * ls;
            const uint8_t *top = row - ls, *top2 = row - 2 * ls;
            // sliding neighbours (FFmpeg's sample-buffer borders: 0 above the
            // slice, L = T at column 0, TL = the row above that's first sample,
            // TR = T past the last column)
            int T = y > 0 ? (a.bytes == 2 ? ldpx<uint16_t>(top, 0) : ldpx<uint8_t>(top, 0)) : 0;
            int TL = y > 1 ? (a.bytes == 2 ? ldpx<uint16_t>(top2, 0) : ldpx<uint8_t>(top2, 0)) : 0;
            int L = T;
            // samples one column ahead are loaded before the current one is
            // coded, so their latency hides behind the range coder
            auto ld = [&](const uint8_t *r, int x) {
                return a.bytes == 2 ? ldpx<uint16_t>(r, x) : ldpx<uint8_t>(r, x);
            };
            // top row two columns ahead (tr1 = TR of the next column), so the
            // next column's context -- and the HBM state block it needs, when
            // it differs from the current one -- is known before this column
            // is coded: the block's load overlaps the range coder
            int nv = ld(row, 0);
            int tr0 = pw > 1 ? (y > 0 ? ld(top, 1) : 0) : T;
            int tr1 = pw > 2 ? (y > 0 ? ld(top, 2) : 0) : tr0;
            int pre_key = -1;
            uint2 pre[4];
            for (int x = 0; x < pw; x++) {
                const int TR = tr0, v = nv;
                if (x + 1 < pw) nv = ld(row, x + 1);
                const int tr2 = x + 3 < pw ? (y > 0 ? ld(top, x + 3) : 0) : tr1;
                int ctx = dquant((L - TL) & 0xFF) + 11 * dquant((TL - T) & 0xFF) + 121 * dquant((T - TR) & 0xFF);
                int diff = v - median3(L, L + T - TL, T);
                if (ctx < 0) {
                    ctx = -ctx;
                    diff = -diff;
                }
                diff &= mask;
                diff = diff >= half ? diff - (mask + 1) : diff;
                const int key = key0 + ctx;
                if (key != cur_key) {
                    if (key == pre_key) {  // prefetched: write the old block back, install the new
                        uint2 *g = reinterpret_cast<uint2 *>(st0 + cur_key * kCtxSize);
                        uint2 *l = reinterpret_cast<uint2 *>(slot);
#pragma unroll
                        for (int i = 0; i < 4; i++) g[i] = l[i];
#pragma unroll
                        for (int i = 0; i < 4; i++) l[i] = pre[i];
                        cur_key = key;
                    } else {
                        switch_ctx(key);
                    }
                }
                // next column: L = v, TL = T, T = TR, TR = tr1
                if (x + 1 < pw) {
                    int c1 = dquant((v - T) & 0xFF) + 11 * dquant((T - TR) & 0xFF) + 121 * dquant((TR - tr1) & 0xFF);
                    const int k1 = key0 + (c1 < 0 ? -c1 : c1);
                    if (k1 != key) {
                        const uint2 *g = reinterpret_cast<const uint2 *>(st0 + k1 * kCtxSize);
#pragma unroll
                        for (int i = 0; i < 4; i++) pre[i] = g[i];
                        pre_key = k1;
                    }
                }
                c.symbol(slot, diff, true);
                tr0 = tr1;
                tr1 = tr2;
                TL = T;
                T = TR;
                L = v;
            }
        }
    }
    hs[33] = 129;  // the closing 0 bit at state 129 (ffv1enc.c encode_frame)
    c.rac(hs + 33, 0);
    c.range = 0xFF;  // ff_rac_terminate: two one-byte flushes
    c.low += 0xFF;
    c.renorm();
    c.range = 0xFF;
    c.renorm();
    const int64_t n = c.p - (a.out + (int64_t)g * a.cap);
    a.sizes[g] = c.over ? -1 : n;
    a.crcs[g] = c.crc;
}

// Frame packets: slice g's bytes at off[g], then its footer: 24-bit size (BE),
// error status 0, CRC-32 parity of everything before it (BE).  One workgroup
// per slice, 16-B copies.
__global__ __launch_bounds__(256) void ffv1_pack_kernel(const uint8_t *slices, int64_t cap, const int64_t *sizes,
                                                        const uint32_t *crcs, const int64_t *off, uint8_t *out,
                                                        const uint32_t *crc_tab) {
    const int g = blockIdx.x;
    const int64_t n = sizes[g];
    const uint8_t *s = slices + (int64_t)g * cap;
    uint8_t *d = out + off[g];
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) d[i] = s[i];
    if (threadIdx.x == 0) {
        uint8_t f[4] = {(uint8_t)(n >> 16), (uint8_t)(n >> 8), (uint8_t)n, 0};
        uint32_t crc = crcs[g];
        for (int i = 0; i < 4; i++) crc = (crc << 8) ^ crc_tab[(crc >> 24) ^ f[i]];
        d[n] = f[0]; d[n + 1] = f[1]; d[n + 2] = f[2]; d[n + 3] = 0;
        d[n + 4] = (uint8_t)(crc >> 24); d[n + 5] = (uint8_t)(crc >> 16);
        d[n + 6] = (uint8_t)(crc >> 8); d[n + 7] = (uint8_t)crc;
    }
}

}  // namespace pp

using namespace pp;

struct pp_ffv1_enc {
    pp_ctx *ctx = nullptr;
    int fmt = 0, w = 0, h = 0, nh = 1, nv = 1, max_frames = 0;
    FmtInfo fi{};
    int64_t cap = 0;           // per-slice output bytes
    uint8_t *slices = nullptr, *states = nullptr, *tables = nullptr;
    int64_t *sizes = nullptr, *off = nullptr;
    uint32_t *crcs = nullptr;
    std::vector<uint8_t> extradata;
};

extern "C" int pp_ffv1_encoder_create(pp_ctx *ctx, int fmt, int w, int h, int slices_h, int slices_v,
                                      int max_frames, pp_ffv1_enc **out) {
    if (!out) PP_FAIL(PP_ERR_INVALID, "null argument");
    *out = nullptr;
    const FmtInfo fi = fmt_info(fmt);
    if (!fi.valid || fi.packed) PP_FAIL(PP_ERR_INVALID, "format %d: planar YUV only", fmt);
    if (w < 2 || h < 2 || w > 16384 || h > 16384) PP_FAIL(PP_ERR_INVALID, "bad size %dx%d", w, h);
    if (slices_h < 1 || slices_v < 1 || slices_h * slices_v > 256 || slices_h > w / 4 || slices_v > h / 4)
        PP_FAIL(PP_ERR_INVALID, "slice grid %dx%d", slices_h, slices_v);
    if (max_frames < 1) PP_FAIL(PP_ERR_INVALID, "max_frames %d", max_frames);
    std::unique_ptr<pp_ffv1_enc> E(new pp_ffv1_enc());
    E->ctx = ctx; E->fmt = fmt; E->w = w; E->h = h; E->nh = slices_h; E->nv = slices_v; E->fi = fi;
    E->max_frames = max_frames;
    // configuration record (RFC 9043 4.2, ffv1enc.c write_extradata)
    {
        HostRC c;
        rac_states(c.zero, c.one);
        uint8_t st[kCtxSize];
        std::memset(st, 128, sizeof(st));
        const int v1[] = {3, 4, 1, 0, fi.depth};  // version, micro_version, coder_type, colorspace, bits
        for (int v : v1) c.symbol(st, v);
        c.rac(st, 1);  // chroma_planes
        c.symbol(st, fi.hsub);
        c.symbol(st, fi.vsub);
        c.rac(st, 0);  // extra_plane
        c.symbol(st, slices_h - 1);
        c.symbol(st, slices_v - 1);
        c.symbol(st, 1);  // quant_table_set_count
        for (int t = 0; t < 5; t++) {
            uint8_t qs[kCtxSize];
            std::memset(qs, 128, sizeof(qs));
            int last = 0, i;
            for (i = 1; i < 128; i++)
                if (t < 3 && quant_host(i) != quant_host(i - 1)) {
                    c.symbol(qs, i - last - 1);
                    last = i;
                }
            c.symbol(qs, i - last - 1);
        }
        c.rac(st, 0);       // states_coded
        c.symbol(st, 1);    // ec
        c.symbol(st, 1);    // intra
        uint8_t s129 = 129;
        c.rac(&s129, 0);
        c.terminate();
        uint32_t t[256];
        crc_table(t);
        uint32_t crc = 0;
        for (uint8_t b : c.out) crc = (crc << 8) ^ t[(crc >> 24) ^ b];
        E->extradata = c.out;
        for (int k = 3; k >= 0; k--) E->extradata.push_back((uint8_t)(crc >> (8 * k)));
    }
    if (!ctx) {  // host-only: configuration record only
        *out = E.release();
        return PP_OK;
    }
    const int per = slices_h * slices_v;
    const int64_t ns = (int64_t)per * max_frames;
    const int sw = (w + slices_h - 1) / slices_h, sh = (h + slices_v - 1) / slices_v;
    const int bytes = fi.depth > 8 ? 2 : 1;
    const int64_t raw = ((int64_t)sw * sh + 2 * (int64_t)((sw + 1) >> fi.hsub) * ((sh + 1) >> fi.vsub)) * bytes;
    E->cap = ((raw * 3 / 2 + 4096) + 255) & ~int64_t(255);  // worst-case expansion is far below 1.5x
    PP_HIP(hipSetDevice(ctx->device));
    PP_HIP(hipMalloc(&E->slices, E->cap * ns));
    PP_HIP(hipMalloc(&E->states, (size_t)kStateBytes * ns));
    PP_HIP(hipMalloc(&E->sizes, sizeof(int64_t) * ns));
    PP_HIP(hipMalloc(&E->off, sizeof(int64_t) * ns));
    PP_HIP(hipMalloc(&E->crcs, sizeof(uint32_t) * ns));
    PP_HIP(hipMalloc(&E->tables, 512 + 1024));
    uint8_t tab[512 + 1024];
    rac_states(tab, tab + 256);
    crc_table(reinterpret_cast<uint32_t *>(tab + 512));
    PP_HIP(hipMemcpy(E->tables, tab, sizeof(tab), hipMemcpyHostToDevice));
    *out = E.release();
    return PP_OK;
}

extern "C" int pp_ffv1_encoder_destroy(pp_ffv1_enc *E) {
    if (!E) return PP_OK;
    for (void *p : {(void *)E->slices, (void *)E->states, (void *)E->sizes, (void *)E->off, (void *)E->crcs,
                    (void *)E->tables})
        if (p) (void)hipFree(p);
    delete E;
    return PP_OK;
}

extern "C" int pp_ffv1_extradata(const pp_ffv1_enc *E, uint8_t *out, int cap) {
    if (!E || (!out && cap)) PP_FAIL(PP_ERR_INVALID, "null argument");
    const int n = (int)E->extradata.size();
    if (out && cap >= n) std::memcpy(out, E->extradata.data(), n);
    return n;
}

extern "C" int64_t pp_ffv1_encode(pp_ffv1_enc *E, const pp_frames *src, int nframes, uint8_t *dst, int64_t dst_cap,
                                  int64_t *frame_sizes, void *stream) {
    if (!E || !src || !dst || !frame_sizes || nframes < 0) PP_FAIL(PP_ERR_INVALID, "null argument");
    if (!E->ctx) PP_FAIL(PP_ERR_INVALID, "host-only encoder cannot encode");
    if (nframes > E->max_frames) PP_FAIL(PP_ERR_INVALID, "%d frames > max_frames %d", nframes, E->max_frames);
    if (nframes == 0) return 0;
    hipStream_t st = static_cast<hipStream_t>(stream);
    PP_HIP(hipSetDevice(E->ctx->device));
    const int per = E->nh * E->nv;
    const int ns = per * nframes;
    Ffv1Args a{};
    for (int p = 0; p < 3; ++p) {
        a.src[p] = static_cast<const uint8_t *>(src->data[p]);
        a.ls[p] = src->linesize[p];
        a.fs[p] = src->frame_stride[p];
    }
    a.w = E->w; a.h = E->h; a.bytes = E->fi.depth > 8 ? 2 : 1; a.bits = E->fi.depth;
    a.hsub = E->fi.hsub; a.vsub = E->fi.vsub; a.nh = E->nh; a.nv = E->nv; a.nslices = ns;
    a.out = E->slices; a.cap = E->cap; a.states = E->states; a.sizes = E->sizes; a.crcs = E->crcs;
    a.tables = E->tables;
    PP_HIP(hipMemsetAsync(E->states, 128, (size_t)kStateBytes * ns, st));  // every context of every slice: 128
    hipLaunchKernelGGL(ffv1_slice_kernel, dim3((ns + 63) / 64), dim3(64), 0, st, a);
    PP_HIP(hipGetLastError());
    std::vector<int64_t> sizes(ns), off(ns);
    PP_HIP(hipMemcpyAsync(sizes.data(), E->sizes, sizeof(int64_t) * ns, hipMemcpyDeviceToHost, st));
    PP_HIP(hipStreamSynchronize(st));
    int64_t total = 0;
    for (int f = 0; f < nframes; ++f) {
        int64_t fsz = 0;
        for (int s = 0; s < per; ++s) {
            const int64_t n = sizes[f * per + s];
            if (n < 0) PP_FAIL(PP_ERR_NOMEM, "frame %d slice %d exceeds its %lld-byte buffer", f, s, (long long)E->cap);
            off[f * per + s] = total + fsz;
            fsz += n + 8;
        }
        frame_sizes[f] = fsz;
        total += fsz;
    }
    if (total > dst_cap) PP_FAIL(PP_ERR_NOMEM, "packets need %lld bytes, dst holds %lld", (long long)total, (long long)dst_cap);
    PP_HIP(hipMemcpyAsync(E->off, off.data(), sizeof(int64_t) * ns, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(ffv1_pack_kernel, dim3(ns), dim3(256), 0, st, E->slices, E->cap, E->sizes, E->crcs, E->off, dst,
                       reinterpret_cast<const uint32_t *>(E->tables + 512));
    PP_HIP(hipGetLastError());
    PP_HIP(hipStreamSynchronize(st));
    return total;
}
