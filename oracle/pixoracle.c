/*
 * oracle/pixoracle.c -- CPU restatement of the reference's raw-frame pixel path.
 *
 *   *** TEST INFRASTRUCTURE ONLY. ***  Only tests/, __graft_entry__.smoke() and
 *   bench.py's cpu_baseline leg may load this library, and only as the checker /
 *   CPU baseline.  The product (processing-chain_amd/pixpath) never links it.
 *
 * What it restates
 * ----------------
 * The reference (pnats2avhd/processing-chain, lib/ffmpeg.py) does all pixel work
 * by building ffmpeg command strings.  The arithmetic therefore lives in the
 * third-party dependency FFmpeg, pinned at 7.0.2 (reference
 * docker/install_ffmpeg.sh:39-41).  FFmpeg's sources are NOT under
 * /root/reference and no ffmpeg binary/library exists in this container or on
 * the GPU box, so this file restates FFmpeg's published algorithms from its
 * source layout (function names cited below) and anchors them on the
 * reference's call sites:
 *
 *   scale=W:H:flags=bicubic         lib/ffmpeg.py:992 (short AVPVS),
 *                                   :1038 (long-test segment), :1213 (mobile CPVS)
 *   scale=W:-2:flags=bicubic        lib/ffmpeg.py:800 (p01 pre-encode downscale)
 *   -pix_fmt <fmt> auto conversion  lib/ffmpeg.py:994, :1048, :1198
 *   pad=...:x=(ow-iw)/2:y=(oh-ih)/2 lib/ffmpeg.py:1183, :1209
 *   -c:v v210 / rawvideo uyvy422    lib/test_config.py:200-215 via lib/ffmpeg.py:1178,1198
 *
 *   FFmpeg function restated                         here
 *   libswscale/utils.c   initFilter()                po_init_filter()
 *   libswscale/utils.c   get_local_pos(), sws_init_context() (xInc, chroma dims,
 *                        filterAlign x86: H=4, V=2)  po_sws_init()
 *   libswscale/swscale.c hScale8To15_c / hScale16To15_c (C reference, the x86
 *                        SIMD versions are bit-identical integer MACs)   hscale_row()
 *   libswscale/output.c  yuv2planeX_8_c, yuv2plane1_8_c,
 *                        yuv2planeX_10_c_template, yuv2plane1_10_c_template,
 *                        yuv2422_X_c_template (uyvy422)                 vscale_*()
 *   libswscale/swscale.c ff_swscale(): ordered dither (ff_dither_8x8_128) when a
 *                        >8-bit source is narrowed to 8 bit, flat 64 otherwise
 *   libswscale/swscale_unscaled.c  yuv422pToUyvyWrapper, planarCopyWrapper
 *   libavfilter/vf_pad.c + drawutils.c  black fill, chroma-grid rounding  po_pad()
 *   libavcodec/v210enc.c v210_enc_10 (CLIP to [4,1019], 6 px / 16 B, 48-px aligned
 *                        stride, zero line padding)                     po_v210_pack()
 *   libavfilter/vf_fps.c output->input frame map (round-to-nearest)     po_fps_map()
 *
 * PARITY STATUS: parity unpinned.  The reference holds no golden pixel vectors
 *  and FFmpeg is unavailable, so these restatements are
 * checked only by the known-answer properties in tests/test_oracle_*.py.
 * The x86 build of FFmpeg replaces yuv2planeX for 8-bit outputs (no
 * SWS_ACCURATE_RND) by an approximate pmulhw kernel; this file follows the C
 * reference, hence the north_star's +-1 LSB tolerance for scaled samples.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -shared -fPIC).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define PO_SWS_BILINEAR 2
#define PO_SWS_BICUBIC 4
#define PO_SWS_LANCZOS 0x200
#define PO_PARAM_DEFAULT 123456.0
#define PO_MAX_REDUCE_CUTOFF 0.002
#define PO_MAXF 64

enum {
    PO_YUV420P = 0, PO_YUV422P = 1, PO_YUV444P = 2,
    PO_YUV420P10 = 3, PO_YUV422P10 = 4, PO_YUV444P10 = 5,
    PO_UYVY422 = 6,
};

static int fmt_depth(int f) { return (f >= PO_YUV420P10 && f <= PO_YUV444P10) ? 10 : 8; }
static int fmt_hsub(int f)
{
    switch (f) {
    case PO_YUV444P: case PO_YUV444P10: return 0;
    default: return 1;
    }
}
static int fmt_vsub(int f) { return (f == PO_YUV420P || f == PO_YUV420P10) ? 1 : 0; }
static int ceil_rshift(int a, int b) { return -((-a) >> b); }

static int av_log2_u(unsigned v)
{
    int n = 0;
    while (v > 1) { v >>= 1; n++; }
    return n;
}

static int64_t rounded_div(int64_t a, int64_t b)
{
    return (a >= 0 ? a + (b >> 1) : a - (b >> 1)) / b;
}

/*
 * initFilter() restatement (libswscale/utils.c, FFmpeg 7.0).  srcFilter /
 * dstFilter are NULL for vf_scale, the cpu is x86 with MMX (filterAlign
 * passed by the caller), SWS_BITEXACT is not set.
 * Writes dstW*(*outSize) coefficients (int16) and dstW positions.
 * Returns 0 or -1 (unsupported/too large).
 */
int po_init_filter(int16_t *outFilter, int32_t *filterPos, int *outSize,
                   int xInc, int srcW, int dstW, int filterAlign, int one,
                   int flags, double param0, double param1, int srcPos, int dstPos)
{
    int i, j, k;
    int filterSize, filter2Size, minFilterSize;
    int64_t *filter = NULL, *filter2 = NULL;
    const int64_t fone = 1LL << (54 - (av_log2_u((unsigned)(srcW / dstW)) < 8 ?
                                       av_log2_u((unsigned)(srcW / dstW)) : 8));

    if (abs(xInc - 0x10000) < 10 && srcPos == dstPos) { /* unscaled */
        filterSize = 1;
        filter = calloc((size_t)dstW * filterSize, sizeof(int64_t));
        if (!filter) return -1;
        for (i = 0; i < dstW; i++) {
            filter[i * filterSize] = fone;
            filterPos[i] = i;
        }
    } else {
        int64_t xDstInSrc;
        int sizeFactor = -1;
        if (flags & PO_SWS_BICUBIC) sizeFactor = 4;
        else if (flags & PO_SWS_BILINEAR) sizeFactor = 2;
        if (flags & PO_SWS_LANCZOS)
            sizeFactor = param0 != PO_PARAM_DEFAULT ? (int)ceil(2 * param0) : 6;
        if (sizeFactor <= 0) return -1;

        if (xInc <= 1 << 16)
            filterSize = 1 + sizeFactor; /* upscale */
        else
            filterSize = 1 + (sizeFactor * srcW + dstW - 1) / dstW;
        if (filterSize > srcW - 2) filterSize = srcW - 2;
        if (filterSize < 1) filterSize = 1;
        if (filterSize > PO_MAXF) return -1;

        filter = malloc((size_t)dstW * filterSize * sizeof(int64_t));
        if (!filter) return -1;
        xDstInSrc = ((dstPos * (int64_t)xInc) >> 7) - ((srcPos * 0x10000LL) >> 7);
        for (i = 0; i < dstW; i++) {
            /* C division: truncation toward zero, as in FFmpeg */
            int xx = (int)((xDstInSrc - (filterSize - 2) * (1LL << 16)) / (1 << 17));
            filterPos[i] = xx;
            for (j = 0; j < filterSize; j++) {
                int64_t d = (llabs(((int64_t)xx * (1 << 17)) - xDstInSrc)) << 13;
                double floatd;
                int64_t coeff;

                if (xInc > 1 << 16)
                    d = d * dstW / srcW;
                floatd = d * (1.0 / (1 << 30));

                if (flags & PO_SWS_BICUBIC) {
                    int64_t B = (int64_t)((param0 != PO_PARAM_DEFAULT ? param0 : 0) * (1 << 24));
                    int64_t C = (int64_t)((param1 != PO_PARAM_DEFAULT ? param1 : 0.6) * (1 << 24));
                    if (d >= 1LL << 31) {
                        coeff = 0;
                    } else {
                        int64_t dd  = (d * d) >> 30;
                        int64_t ddd = (dd * d) >> 30;
                        if (d < 1LL << 30)
                            coeff = (12 * (1 << 24) - 9 * B - 6 * C) * ddd +
                                    (-18 * (1 << 24) + 12 * B + 6 * C) * dd +
                                    (6 * (1 << 24) - 2 * B) * (1 << 30);
                        else
                            coeff = (-B - 6 * C) * ddd +
                                    (6 * B + 30 * C) * dd +
                                    (-12 * B - 48 * C) * d +
                                    (8 * B + 24 * C) * (1 << 30);
                    }
                    coeff /= (1LL << 54) / fone;
                } else if (flags & PO_SWS_LANCZOS) {
                    double p = param0 != PO_PARAM_DEFAULT ? param0 : 3;
                    coeff = (int64_t)((d ? sin(floatd * M_PI) * sin(floatd * M_PI / p) /
                                           (floatd * floatd * M_PI * M_PI / p) : 1.0) * fone);
                    if (floatd > p)
                        coeff = 0;
                } else { /* bilinear */
                    coeff = (1 << 30) - d;
                    if (coeff < 0) coeff = 0;
                    coeff *= fone >> 30;
                }
                filter[i * filterSize + j] = coeff;
                xx++;
            }
            xDstInSrc += 2LL * xInc;
        }
    }

    /* apply src & dst filter: none -> plain copy */
    filter2Size = filterSize;
    filter2 = calloc((size_t)dstW * filter2Size, sizeof(int64_t));
    if (!filter2) { free(filter); return -1; }
    for (i = 0; i < dstW; i++)
        for (j = 0; j < filterSize; j++)
            filter2[i * filter2Size + j] = filter[i * filterSize + j];
    free(filter);
    filter = NULL;

    /* try to reduce the filter-size (step1 find size and shift left) */
    minFilterSize = 0;
    for (i = dstW - 1; i >= 0; i--) {
        int min = filter2Size;
        int64_t cutOff = 0;
        for (j = 0; j < filter2Size; j++) {
            cutOff += llabs(filter2[i * filter2Size]);
            if (cutOff > PO_MAX_REDUCE_CUTOFF * fone)
                break;
            if (i < dstW - 1 && filterPos[i] >= filterPos[i + 1])
                break;
            for (k = 1; k < filter2Size; k++)
                filter2[i * filter2Size + k - 1] = filter2[i * filter2Size + k];
            filter2[i * filter2Size + k - 1] = 0;
            filterPos[i]++;
        }
        cutOff = 0;
        for (j = filter2Size - 1; j > 0; j--) {
            cutOff += llabs(filter2[i * filter2Size + j]);
            if (cutOff > PO_MAX_REDUCE_CUTOFF * fone)
                break;
            min--;
        }
        if (min > minFilterSize)
            minFilterSize = min;
    }

    /* x86 MMX: special case for unscaled vertical filtering */
    if (minFilterSize == 1 && filterAlign == 2)
        filterAlign = 1;
    filterSize = (minFilterSize + (filterAlign - 1)) & (~(filterAlign - 1));
    if (filterSize > PO_MAXF) { free(filter2); return -1; }
    filter = malloc((size_t)dstW * filterSize * sizeof(int64_t));
    if (!filter) { free(filter2); return -1; }
    *outSize = filterSize;

    /* step2: reduce it */
    for (i = 0; i < dstW; i++)
        for (j = 0; j < filterSize; j++)
            filter[i * filterSize + j] = j >= filter2Size ? 0 : filter2[i * filter2Size + j];
    free(filter2);

    /* fix borders */
    for (i = 0; i < dstW; i++) {
        if (filterPos[i] < 0) {
            for (j = 1; j < filterSize; j++) {
                int left = j + filterPos[i] > 0 ? j + filterPos[i] : 0;
                filter[i * filterSize + left] += filter[i * filterSize + j];
                filter[i * filterSize + j] = 0;
            }
            filterPos[i] = 0;
        }
        if (filterPos[i] + filterSize > srcW) {
            int shift = filterPos[i] + (filterSize - srcW < 0 ? filterSize - srcW : 0);
            int64_t acc = 0;
            for (j = filterSize - 1; j >= 0; j--) {
                if (filterPos[i] + j >= srcW) {
                    acc += filter[i * filterSize + j];
                    filter[i * filterSize + j] = 0;
                }
            }
            for (j = filterSize - 1; j >= 0; j--) {
                if (j < shift)
                    filter[i * filterSize + j] = 0;
                else
                    filter[i * filterSize + j] = filter[i * filterSize + j - shift];
            }
            filterPos[i] -= shift;
            filter[i * filterSize + srcW - 1 - filterPos[i]] += acc;
        }
    }

    /* normalize & store in outFilter (error diffusion) */
    for (i = 0; i < dstW; i++) {
        int64_t error = 0, sum = 0;
        for (j = 0; j < filterSize; j++)
            sum += filter[i * filterSize + j];
        sum = (sum + one / 2) / one;
        if (!sum) sum = 1;
        for (j = 0; j < filterSize; j++) {
            int64_t v = filter[i * filterSize + j] + error;
            int intV = (int)rounded_div(v, sum);
            outFilter[i * filterSize + j] = (int16_t)intV;
            error = v - intV * sum;
        }
    }
    free(filter);
    return 0;
}

/* get_local_pos() (libswscale/utils.c): chroma sample position in 1/256 px. */
static int get_local_pos(int chr_subsample, int pos)
{
    if (pos == -1 || pos <= -513)
        pos = (128 << chr_subsample) - 128;
    pos += 128;
    return pos >> chr_subsample;
}

typedef struct po_filter {
    int size;
    int16_t *coef; /* n * size */
    int32_t *pos;  /* n */
} po_filter;

typedef struct po_sws {
    int src_fmt, dst_fmt, sw, sh, dw, dh;
    int csw, csh, cdw, cdh;
    int src_depth, dst_depth;
    po_filter hl, hc, vl, vc;
    int kind; /* 0 generic, 1 copy/widen, 2 interleave 422p->uyvy */
} po_sws;

static int make_filter(po_filter *f, int inc, int srcW, int dstW, int align, int one,
                       int flags, double p0, double p1, int sp, int dp)
{
    int16_t *tmp = malloc((size_t)dstW * PO_MAXF * sizeof(int16_t));
    f->pos = malloc((size_t)dstW * sizeof(int32_t));
    if (!tmp || !f->pos) return -1;
    if (po_init_filter(tmp, f->pos, &f->size, inc, srcW, dstW, align, one, flags, p0, p1, sp, dp))
        return -1;
    f->coef = malloc((size_t)dstW * f->size * sizeof(int16_t));
    memcpy(f->coef, tmp, (size_t)dstW * f->size * sizeof(int16_t));
    free(tmp);
    return 0;
}

void po_sws_free(po_sws *c)
{
    if (!c) return;
    free(c->hl.coef); free(c->hl.pos); free(c->hc.coef); free(c->hc.pos);
    free(c->vl.coef); free(c->vl.pos); free(c->vc.coef); free(c->vc.pos);
    free(c);
}

/*
 * sws_init_context() restatement for planar YUV in / planar YUV or uyvy422 out.
 * chr positions default to -513 (vf_scale defaults; its yuv420p override to
 * 128 yields the same local position).  Returns NULL when unsupported.
 */
po_sws *po_sws_init(int src_fmt, int sw, int sh, int dst_fmt, int dw, int dh,
                    int flags, double p0, double p1)
{
    po_sws *c = calloc(1, sizeof(*c));
    int dst_hsub, dst_vsub, lumXInc, lumYInc, chrXInc, chrYInc;
    if (!c) return NULL;
    c->src_fmt = src_fmt; c->dst_fmt = dst_fmt;
    c->sw = sw; c->sh = sh; c->dw = dw; c->dh = dh;
    c->src_depth = fmt_depth(src_fmt);
    c->dst_depth = dst_fmt == PO_UYVY422 ? 8 : fmt_depth(dst_fmt);
    dst_hsub = dst_fmt == PO_UYVY422 ? 1 : fmt_hsub(dst_fmt);
    dst_vsub = dst_fmt == PO_UYVY422 ? 0 : fmt_vsub(dst_fmt);
    c->csw = ceil_rshift(sw, fmt_hsub(src_fmt));
    c->csh = ceil_rshift(sh, fmt_vsub(src_fmt));
    c->cdw = ceil_rshift(dw, dst_hsub);
    c->cdh = ceil_rshift(dh, dst_vsub);

    /* unscaled special converters (ff_get_unscaled_swscale) */
    if (sw == dw && sh == dh) {
        if (src_fmt == PO_YUV422P && dst_fmt == PO_UYVY422) { c->kind = 2; return c; }
        if (dst_fmt != PO_UYVY422 && fmt_hsub(src_fmt) == dst_hsub &&
            fmt_vsub(src_fmt) == dst_vsub && c->src_depth <= c->dst_depth) {
            c->kind = 1; /* planarCopyWrapper: copy or 8->10 shift */
            return c;
        }
    }
    c->kind = 0;
    lumXInc = (int)((((int64_t)sw << 16) + (dw >> 1)) / dw);
    lumYInc = (int)((((int64_t)sh << 16) + (dh >> 1)) / dh);
    chrXInc = (int)((((int64_t)c->csw << 16) + (c->cdw >> 1)) / c->cdw);
    chrYInc = (int)((((int64_t)c->csh << 16) + (c->cdh >> 1)) / c->cdh);
    if (make_filter(&c->hl, lumXInc, sw, dw, 4, 1 << 14, flags, p0, p1,
                    get_local_pos(0, -513), get_local_pos(0, -513)) ||
        make_filter(&c->hc, chrXInc, c->csw, c->cdw, 4, 1 << 14, flags, p0, p1,
                    get_local_pos(fmt_hsub(src_fmt), -513), get_local_pos(dst_hsub, -513)) ||
        make_filter(&c->vl, lumYInc, sh, dh, 2, 1 << 12, flags, p0, p1,
                    get_local_pos(0, -513), get_local_pos(0, -513)) ||
        make_filter(&c->vc, chrYInc, c->csh, c->cdh, 2, 1 << 12, flags, p0, p1,
                    get_local_pos(fmt_vsub(src_fmt), -513), get_local_pos(dst_vsub, -513))) {
        po_sws_free(c);
        return NULL;
    }
    return c;
}

int po_sws_filter_size(const po_sws *c, int which)
{
    const po_filter *f = which == 0 ? &c->hl : which == 1 ? &c->hc : which == 2 ? &c->vl : &c->vc;
    return c->kind ? 0 : f->size;
}

/* Copy one filter (0 hl, 1 hc, 2 vl, 3 vc) out for introspection. */
int po_sws_get_filter(const po_sws *c, int which, int16_t *coef, int32_t *pos)
{
    const po_filter *f = which == 0 ? &c->hl : which == 1 ? &c->hc : which == 2 ? &c->vl : &c->vc;
    int n = which == 0 ? c->dw : which == 1 ? c->cdw : which == 2 ? c->dh : c->cdh;
    if (c->kind) return -1;
    memcpy(coef, f->coef, (size_t)n * f->size * sizeof(int16_t));
    memcpy(pos, f->pos, (size_t)n * sizeof(int32_t));
    return f->size;
}

/* ff_dither_8x8_128 (libswscale/swscale.c) */
static const uint8_t dither_8x8_128[9][8] = {
    {  36, 68,  60, 92,  34, 66,  58, 90, },
    { 100,  4, 124, 28,  98,  2, 122, 26, },
    {  52, 84,  44, 76,  50, 82,  42, 74, },
    { 116, 20, 108, 12, 114, 18, 106, 10, },
    {  32, 64,  56, 88,  38, 70,  62, 94, },
    {  96,  0, 120, 24, 102,  6, 126, 30, },
    {  48, 80,  40, 72,  54, 86,  46, 78, },
    { 112, 16, 104,  8, 118, 22, 110, 14, },
    {  36, 68,  60, 92,  34, 66,  58, 90, },
};
static const uint8_t flat64[8] = { 64, 64, 64, 64, 64, 64, 64, 64 };

/* hScale8To15_c / hScale16To15_c: one source row -> 15-bit intermediates */
static void hscale_row(int16_t *dst, int dstW, const uint8_t *src8, const uint16_t *src16,
                       int depth, const po_filter *f)
{
    int sh = depth - 1;
    for (int i = 0; i < dstW; i++) {
        int p = f->pos[i], val = 0;
        for (int j = 0; j < f->size; j++) {
            int s = src8 ? src8[p + j] : src16[p + j];
            val += s * f->coef[f->size * i + j];
        }
        val = src8 ? val >> 7 : val >> sh;
        dst[i] = (int16_t)(val < (1 << 15) - 1 ? val : (1 << 15) - 1);
    }
}

static inline int clip_u8(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }
static inline int clip_u10(int v) { return v < 0 ? 0 : v > 1023 ? 1023 : v; }

/*
 * Vertical pass for one output row of one plane.  rows[] holds intermediates for
 * the source rows [pos, pos+size).  Writes either an 8-bit or 10-bit planar row.
 */
static void vscale_row(void *dst, int dstW, int16_t *const *rows, const int16_t *coef,
                       int size, int dst_depth, const uint8_t *dither, int offset)
{
    if (dst_depth == 8) {
        uint8_t *d = dst;
        if (size == 1) { /* yuv2plane1_8_c */
            for (int i = 0; i < dstW; i++)
                d[i] = (uint8_t)clip_u8((rows[0][i] + dither[(i + offset) & 7]) >> 7);
        } else { /* yuv2planeX_8_c */
            for (int i = 0; i < dstW; i++) {
                int val = dither[(i + offset) & 7] << 12;
                for (int j = 0; j < size; j++)
                    val += rows[j][i] * coef[j];
                d[i] = (uint8_t)clip_u8(val >> 19);
            }
        }
    } else {
        uint16_t *d = dst;
        if (size == 1) { /* yuv2plane1_10_c_template: shift = 15 - 10 */
            for (int i = 0; i < dstW; i++)
                d[i] = (uint16_t)clip_u10((rows[0][i] + (1 << 4)) >> 5);
        } else { /* yuv2planeX_10_c_template: shift = 11 + 16 - 10 */
            for (int i = 0; i < dstW; i++) {
                int val = 1 << 16;
                for (int j = 0; j < size; j++)
                    val += rows[j][i] * coef[j];
                d[i] = (uint16_t)clip_u10(val >> 17);
            }
        }
    }
}

/* Scale one plane through the generic H->V pipeline. */
static int scale_plane(const uint8_t *src, int64_t sls, int sw, int sh, int sdepth,
                       uint8_t *dst, int64_t dls, int dw, int dh, int ddepth,
                       const po_filter *hf, const po_filter *vf, int dither_on, int offset)
{
    int16_t *inter = malloc((size_t)sh * dw * sizeof(int16_t));
    int16_t *rows[PO_MAXF];
    (void)sw;
    if (!inter) return -1;
    for (int y = 0; y < sh; y++) {
        const uint8_t *row = src + (int64_t)y * sls;
        hscale_row(inter + (size_t)y * dw, dw, sdepth == 8 ? row : NULL,
                   sdepth == 8 ? NULL : (const uint16_t *)row, sdepth, hf);
    }
    for (int y = 0; y < dh; y++) {
        for (int j = 0; j < vf->size; j++)
            rows[j] = inter + (size_t)(vf->pos[y] + j) * dw;
        vscale_row(dst + (int64_t)y * dls, dw, rows, vf->coef + (size_t)y * vf->size,
                   vf->size, ddepth, dither_on ? dither_8x8_128[y & 7] : flat64, offset);
    }
    free(inter);
    return 0;
}

/*
 * Full conversion of one frame.  src/dst: plane pointers and byte linesizes.
 * For uyvy422 output only dst[0]/dls[0] are used.
 */
int po_sws_scale(const po_sws *c, const uint8_t *const src[3], const int64_t sls[3],
                 uint8_t *const dst[3], const int64_t dls[3])
{
    if (c->kind == 2) { /* yuv422pToUyvyWrapper -> yuvPlanartouyvy_c */
        for (int y = 0; y < c->sh; y++) {
            const uint8_t *Y = src[0] + y * sls[0], *U = src[1] + y * sls[1], *V = src[2] + y * sls[2];
            uint8_t *d = dst[0] + y * dls[0];
            for (int x = 0; x < (c->sw + 1) / 2; x++) {
                d[4 * x + 0] = U[x];
                d[4 * x + 1] = Y[2 * x];
                d[4 * x + 2] = V[x];
                d[4 * x + 3] = Y[2 * x + 1];
            }
        }
        return 0;
    }
    if (c->kind == 1) { /* planarCopyWrapper, limited range: shift only */
        int sh = c->dst_depth - c->src_depth;
        for (int p = 0; p < 3; p++) {
            int w = p ? c->csw : c->sw, h = p ? c->csh : c->sh;
            for (int y = 0; y < h; y++) {
                const uint8_t *s = src[p] + y * sls[p];
                uint8_t *d = dst[p] + y * dls[p];
                for (int x = 0; x < w; x++) {
                    int v = c->src_depth == 8 ? s[x] : ((const uint16_t *)s)[x];
                    if (c->dst_depth == 8) d[x] = (uint8_t)v;
                    else ((uint16_t *)d)[x] = (uint16_t)(v << sh);
                }
            }
        }
        return 0;
    }
    const int dith = c->src_depth > 8 && c->dst_depth == 8;
    if (c->dst_fmt != PO_UYVY422) {
        if (scale_plane(src[0], sls[0], c->sw, c->sh, c->src_depth, dst[0], dls[0], c->dw, c->dh,
                        c->dst_depth, &c->hl, &c->vl, dith, 0) ||
            scale_plane(src[1], sls[1], c->csw, c->csh, c->src_depth, dst[1], dls[1], c->cdw, c->cdh,
                        c->dst_depth, &c->hc, &c->vc, dith, 0) ||
            scale_plane(src[2], sls[2], c->csw, c->csh, c->src_depth, dst[2], dls[2], c->cdw, c->cdh,
                        c->dst_depth, &c->hc, &c->vc, dith, 3))
            return -1;
        return 0;
    }
    /* uyvy422 through yuv2packedX (yuv2422_X_c_template): planes are filtered
     * with the same H/V tables, rounding constant 1<<18 (no dither) */
    {
        int64_t pl[3] = { c->dw, c->cdw, c->cdw };
        uint8_t *tmp[3];
        int64_t tls[3];
        int rc = 0;
        for (int p = 0; p < 3; p++) {
            tls[p] = pl[p];
            tmp[p] = malloc((size_t)pl[p] * c->dh);
        }
        rc |= scale_plane(src[0], sls[0], c->sw, c->sh, c->src_depth, tmp[0], tls[0], c->dw, c->dh,
                          8, &c->hl, &c->vl, 0, 0);
        rc |= scale_plane(src[1], sls[1], c->csw, c->csh, c->src_depth, tmp[1], tls[1], c->cdw, c->cdh,
                          8, &c->hc, &c->vc, 0, 0);
        rc |= scale_plane(src[2], sls[2], c->csw, c->csh, c->src_depth, tmp[2], tls[2], c->cdw, c->cdh,
                          8, &c->hc, &c->vc, 0, 3);
        for (int y = 0; y < c->dh && !rc; y++) {
            uint8_t *d = dst[0] + y * dls[0];
            for (int x = 0; x < (c->dw + 1) / 2; x++) {
                d[4 * x + 0] = tmp[1][y * tls[1] + x];
                d[4 * x + 1] = tmp[0][y * tls[0] + 2 * x];
                d[4 * x + 2] = tmp[2][y * tls[2] + x];
                d[4 * x + 3] = (2 * x + 1 < c->dw) ? tmp[0][y * tls[0] + 2 * x + 1] : 0;
            }
        }
        for (int p = 0; p < 3; p++) free(tmp[p]);
        return rc;
    }
}

/*
 * vf_pad (libavfilter/vf_pad.c): copy the input into a black canvas at (x, y).
 * x, y are the already-evaluated offsets; they are rounded down to the chroma
 * grid (ff_draw_round_to_sub, dir -1).  Black: Y 16, C 128, scaled by 2^(d-8).
 */
int po_pad(int fmt, const uint8_t *const src[3], const int64_t sls[3], int sw, int sh,
           uint8_t *const dst[3], const int64_t dls[3], int dw, int dh, int x, int y)
{
    int depth = fmt_depth(fmt), hs = fmt_hsub(fmt), vs = fmt_vsub(fmt), bps = depth > 8 ? 2 : 1;
    x = (x >> hs) << hs;
    y = (y >> vs) << vs;
    if (x < 0 || y < 0 || x + sw > dw || y + sh > dh) return -1;
    for (int p = 0; p < 3; p++) {
        int ps = p ? hs : 0, pv = p ? vs : 0;
        int W = ceil_rshift(dw, ps), H = ceil_rshift(dh, pv);
        int iw = ceil_rshift(sw, ps), ih = ceil_rshift(sh, pv);
        int ox = x >> ps, oy = y >> pv;
        int black = (p ? 128 : 16) << (depth - 8);
        for (int yy = 0; yy < H; yy++) {
            uint8_t *d = dst[p] + yy * dls[p];
            for (int xx = 0; xx < W; xx++) {
                int v = black;
                if (yy >= oy && yy < oy + ih && xx >= ox && xx < ox + iw) {
                    const uint8_t *s = src[p] + (yy - oy) * sls[p];
                    v = bps == 1 ? s[xx - ox] : ((const uint16_t *)s)[xx - ox];
                }
                if (bps == 1) d[xx] = (uint8_t)v; else ((uint16_t *)d)[xx] = (uint16_t)v;
            }
        }
    }
    return 0;
}

/* libavcodec/v210enc.c: bytes per line */
int64_t po_v210_linesize(int w) { return (int64_t)((w + 47) / 48) * 48 * 8 / 3; }

static inline uint32_t v210_clip(int v) { return (uint32_t)(v < 4 ? 4 : v > 1019 ? 1019 : v); }

/* v210_enc_10 over one frame of yuv422p10le. */
int po_v210_pack(const uint16_t *Y, int64_t yls, const uint16_t *U, int64_t uls,
                 const uint16_t *V, int64_t vls, int w, int h, uint8_t *dst, int64_t dls)
{
    int64_t stride = po_v210_linesize(w);
    for (int row = 0; row < h; row++) {
        const uint16_t *y = (const uint16_t *)((const uint8_t *)Y + row * yls);
        const uint16_t *u = (const uint16_t *)((const uint8_t *)U + row * uls);
        const uint16_t *v = (const uint16_t *)((const uint8_t *)V + row * vls);
        uint8_t *d = dst + row * dls, *d0 = d;
        uint32_t val = 0;
        int x;
#define WR(a, b, c) do { val = v210_clip(*a++); val |= (v210_clip(*b++) << 10) | (v210_clip(*c++) << 20); \
                         d[0] = val; d[1] = val >> 8; d[2] = val >> 16; d[3] = val >> 24; d += 4; } while (0)
        for (x = 0; x < w - 5; x += 6) {
            WR(u, y, v);
            WR(y, u, y);
            WR(v, y, u);
            WR(y, v, y);
        }
        if (x < w - 1) {
            WR(u, y, v);
            val = v210_clip(*y++);
            if (x == w - 2) {
                d[0] = val; d[1] = val >> 8; d[2] = val >> 16; d[3] = val >> 24; d += 4;
            }
        }
        if (x < w - 3) {
            val |= (v210_clip(*u++) << 10) | (v210_clip(*y++) << 20);
            d[0] = val; d[1] = val >> 8; d[2] = val >> 16; d[3] = val >> 24; d += 4;
            val = v210_clip(*v++) | (v210_clip(*y++) << 10);
            d[0] = val; d[1] = val >> 8; d[2] = val >> 16; d[3] = val >> 24; d += 4;
        }
#undef WR
        memset(d, 0, (size_t)(stride - (d - d0)));
    }
    return 0;
}

/*
 * vf_fps output->input mapping (libavfilter/vf_fps.c, rounding "near"):
 * output frame k shows the last input frame i whose timestamp, rescaled to
 * the output rate with round-half-away-from-zero, is <= k.  The output length
 * is round(n_in * out_rate / in_rate) (EOF handling, eof_action=round).
 * Rates are given as num/den.  Returns the number of output frames written.
 */
int po_fps_map(int n_in, int64_t in_num, int64_t in_den, int64_t out_num, int64_t out_den,
               int32_t *map, int cap)
{
    /* t_i(out units) = i * in_den * out_num / (in_num * out_den) */
    int64_t N = in_den * out_num, D = in_num * out_den;
    int64_t n_out = (n_in * N + D / 2) / D;
    int i = 0;
    if (n_out > cap) return -1;
    for (int64_t k = 0; k < n_out; k++) {
        while (i + 1 < n_in && ((int64_t)(i + 1) * N * 2 + D) / (2 * D) <= k)
            i++;
        map[k] = i;
    }
    return (int)n_out;
}

/*
 * Timing helper for bench.py's cpu_baseline leg: po_sws_scale of one frame
 * `count` times in one call, so a Python thread per core spends its time in C
 * (the GIL is released for the whole call by ctypes).  Returns 0 or the first
 * failure.
 */
int po_sws_scale_n(const po_sws *c, const uint8_t *const src[3], const int64_t sls[3],
                   uint8_t *const dst[3], const int64_t dls[3], int count)
{
    for (int i = 0; i < count; i++) {
        int rc = po_sws_scale(c, src, sls, dst, dls);
        if (rc) return rc;
    }
    return 0;
}
