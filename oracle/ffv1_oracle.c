/*
 * CPU oracle (TEST INFRASTRUCTURE ONLY -- loaded by tests/ and bench.py's
 * cpu_baseline, never by the product) for the FFV1 AVPVS intermediate
 * (SURVEY.md section 8f row 1): the reference encodes every AVPVS with
 * `-c:v ffv1 -threads 4 -level 3 -coder 1 -context 1 -slicecrc 1`
 * (/root/reference/lib/ffmpeg.py:993, :1047).
 *
 * FFV1 is third-party (FFmpeg 7.0.2 ffv1enc.c / ffv1dec.c / rangecoder.c,
 * specified by RFC 9043); neither FFmpeg nor any FFV1 decoder exists in this
 * container or on the GPU box, so this restatement is PARITY UNPINNED against
 * FFmpeg: it is checked only by its own encoder -> decoder round trip.
 *
 * What is restated (RFC 9043 section, FFmpeg function):
 *   range coder            3.8.1   rangecoder.c ff_init_range_encoder, put_rac /
 *                                  renorm_encoder, ff_rac_terminate (2-step flush),
 *                                  ff_build_rac_states(0.05 * 2^32, 256 - 8)
 *   put_symbol/get_symbol  3.8.1.2 ffv1enc.c put_symbol_inline (32-byte states)
 *   configuration record   4.2     ffv1enc.c write_extradata: version 3,
 *                                  micro_version 4, CRC-32 parity
 *   quantization tables    4.3     write_quant_table (run lengths)
 *   frame / slices         4.4-4.8 keyframe bit, slice header, plane-by-plane
 *                                  content, footer (24-bit size, error status,
 *                                  CRC-32 parity)
 *   samples / context      3.1-3.5 ffv1enc.c encode_plane / encode_line:
 *                                  median prediction, 3-input context, fold
 *
 * Encoder choices that differ from `ffmpeg -c:v ffv1 -level 3 -coder 1
 * -context 1 -slicecrc 1` (a decoder reads all of them from the bitstream,
 * so decoded pixels are unaffected; the bitstream bytes differ):
 *   - coder_type 1 (range coder, default state table) instead of FFmpeg's
 *     transmitted custom table (coder_type 2, ver2_state -- not available here);
 *   - one quantization table set of 3 inputs, a threshold quantiser per
 *     bit depth (oracle_quant: 63 contexts at 10 bits, 172 at 8) instead of
 *     -context 1's 5-input set;
 *   - every frame a keyframe (intra = 1; FFmpeg's default GOP of 12 carries
 *     context state from frame to frame, which would serialise frames);
 *   - num_h_slices x num_v_slices chosen by the caller (FFmpeg: 2 x 2 for
 *     -threads 4).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define CTX_SIZE 32
#define NCTX 666  /* (11 * 11 * 11 + 1) / 2: the most contexts a pixpath quantiser has */

/* ---- range coder (rangecoder.c) ---------------------------------------- */
typedef struct {
    int low, range, outstanding_count, outstanding_byte;
    uint8_t zero_state[256], one_state[256];
    uint8_t *buf, *p, *end;
    int overflow;
} RC;

static void build_states(RC *c) {
    const int64_t one = (int64_t)1 << 32;
    const int64_t factor = (int64_t)(0.05 * (double)((int64_t)1 << 32));
    const int max_p = 256 - 8;
    int64_t p;
    int last_p8 = 0, p8, i;
    memset(c->zero_state, 0, 256);
    memset(c->one_state, 0, 256);
    p = one / 2;
    for (i = 0; i < 128; i++) {
        p8 = (int)((256 * p + one / 2) >> 32);
        if (p8 <= last_p8) p8 = last_p8 + 1;
        if (last_p8 && last_p8 < 256 && p8 <= max_p) c->one_state[last_p8] = (uint8_t)p8;
        p += ((one - p) * factor + one / 2) >> 32;
        last_p8 = p8;
    }
    for (i = 256 - max_p; i <= max_p; i++) {
        if (c->one_state[i]) continue;
        p = (i * one + 128) >> 8;
        p += ((one - p) * factor + one / 2) >> 32;
        p8 = (int)((256 * p + one / 2) >> 32);
        if (p8 <= i) p8 = i + 1;
        if (p8 > max_p) p8 = max_p;
        c->one_state[i] = (uint8_t)p8;
    }
    for (i = 1; i < 255; i++) c->zero_state[i] = (uint8_t)(256 - c->one_state[256 - i]);
}

void ffv1o_state_tables(uint8_t *zero, uint8_t *one) {
    RC c;
    build_states(&c);
    memcpy(zero, c.zero_state, 256);
    memcpy(one, c.one_state, 256);
}

static void rc_init(RC *c, uint8_t *buf, int64_t cap) {
    c->low = 0;
    c->range = 0xFF00;
    c->outstanding_count = 0;
    c->outstanding_byte = -1;
    c->buf = c->p = buf;
    c->end = buf + cap;
    c->overflow = 0;
}

static void out_byte(RC *c, int v) {
    if (c->p < c->end) *c->p++ = (uint8_t)v;
    else c->overflow = 1;
}

static void renorm(RC *c) {
    while (c->range < 0x100) {
        if (c->outstanding_byte < 0) {
            c->outstanding_byte = c->low >> 8;
        } else if (c->low <= 0xFF00) {
            out_byte(c, c->outstanding_byte);
            for (; c->outstanding_count; c->outstanding_count--) out_byte(c, 0xFF);
            c->outstanding_byte = c->low >> 8;
        } else if (c->low >= 0x10000) {
            out_byte(c, c->outstanding_byte + 1);
            for (; c->outstanding_count; c->outstanding_count--) out_byte(c, 0x00);
            c->outstanding_byte = (c->low >> 8) - 0x100;
        } else {
            c->outstanding_count++;
        }
        c->low = (c->low & 0xFF) << 8;
        c->range <<= 8;
    }
}

static void put_rac(RC *c, uint8_t *state, int bit) {
    const int range1 = (c->range * (*state)) >> 8;
    if (!bit) {
        c->range -= range1;
        *state = c->zero_state[*state];
    } else {
        c->low += c->range - range1;
        c->range = range1;
        *state = c->one_state[*state];
    }
    renorm(c);
}

static int64_t rc_terminate(RC *c) {
    c->range = 0xFF;
    c->low += 0xFF;
    renorm(c);
    c->range = 0xFF;
    renorm(c);
    return c->p - c->buf;
}

static int log2i(unsigned v) {
    int n = 0;
    while (v >>= 1) n++;
    return n;
}

static void put_symbol(RC *c, uint8_t *state, int v, int is_signed) {
    int i;
    if (v) {
        const int a = v < 0 ? -v : v;
        const int e = log2i((unsigned)a);
        put_rac(c, state + 0, 0);
        for (i = 0; i < e; i++) put_rac(c, state + 1 + (i < 9 ? i : 9), 1);
        put_rac(c, state + 1 + (e < 9 ? e : 9), 0);
        for (i = e - 1; i >= 0; i--) put_rac(c, state + 22 + (i < 9 ? i : 9), (a >> i) & 1);
        if (is_signed) put_rac(c, state + 11 + (e < 10 ? e : 10), v < 0);
    } else {
        put_rac(c, state + 0, 1);
    }
}

/* ---- range decoder ------------------------------------------------------ */
typedef struct {
    int low, range;
    uint8_t zero_state[256], one_state[256];
    const uint8_t *p, *end;
    int overread;
} RD;

static void rd_init(RD *d, const uint8_t *buf, int64_t size) {
    RC tmp;
    build_states(&tmp);
    memcpy(d->zero_state, tmp.zero_state, 256);
    memcpy(d->one_state, tmp.one_state, 256);
    d->p = buf;
    d->end = buf + size;
    d->range = 0xFF00;
    d->low = size >= 2 ? (buf[0] << 8) | buf[1] : 0;
    d->p += 2;
    d->overread = 0;
    if (d->low >= 0xFF00) { d->low = 0xFF00; d->end = d->p; }
}

static void refill(RD *d) {
    if (d->range < 0x100) {
        d->range <<= 8;
        d->low <<= 8;
        if (d->p < d->end) d->low += *d->p++;
        else d->overread++;
    }
}

static int get_rac(RD *d, uint8_t *state) {
    const int range1 = (d->range * (*state)) >> 8;
    d->range -= range1;
    if (d->low < d->range) {
        *state = d->zero_state[*state];
        refill(d);
        return 0;
    }
    d->low -= d->range;
    *state = d->one_state[*state];
    d->range = range1;
    refill(d);
    return 1;
}

static int get_symbol(RD *d, uint8_t *state, int is_signed) {
    if (get_rac(d, state + 0)) return 0;
    int e = 0, i, a;
    while (get_rac(d, state + 1 + (e < 9 ? e : 9))) {
        e++;
        if (e > 31) return 0x7fffffff;
    }
    a = 1;
    for (i = e - 1; i >= 0; i--) a += a + get_rac(d, state + 22 + (i < 9 ? i : 9));
    return (is_signed && get_rac(d, state + 11 + (e < 10 ? e : 10))) ? -a : a;
}

/* ---- CRC-32 (AV_CRC_32_IEEE: poly 0x04C11DB7, MSB first, init 0, no xor) */
static uint32_t crc_table[256];
static int crc_ready;
static void crc_init(void) {
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i << 24;
        for (int j = 0; j < 8; j++) c = (c << 1) ^ ((c & 0x80000000u) ? 0x04C11DB7u : 0);
        crc_table[i] = c;
    }
    crc_ready = 1;
}
uint32_t ffv1o_crc(uint32_t crc, const uint8_t *p, int64_t n) {
    if (!crc_ready) crc_init();
    for (int64_t i = 0; i < n; i++) crc = (crc << 8) ^ crc_table[(crc >> 24) ^ p[i]];
    return crc;
}
static void put_be32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}

/* ---- quantisation (ffv1host.cpp Ffv1Quant): the level of |d| is the number
 * of thresholds <= |d|, on (d & 0xFF) as int8.  The thresholds the encoder
 * uses for a bit depth (ffv1host.cpp ffv1_default_quant): */
typedef struct { int n, thr[5]; } Quant;
static Quant oracle_quant(int bits) {
    /* 10 bits: thresholds 4, 32 (5 levels, 63 contexts); 8 bits: 1, 3, 8
     * (7 levels, 172 contexts).  Round 4's encoder used 1, 2, 4, 8, 16 =
     * min(5, bit length |d|) (11 levels, 666 contexts) at every depth. */
    Quant q10 = {2, {4, 32}}, q8 = {3, {1, 3, 8}};
    return bits > 8 ? q10 : q8;
}
static int levels(const Quant *q) { return 2 * q->n + 1; }

static int quant_q(const Quant *q, int i /* 0..255 */) {
    if (i < 128) {
        int lv = 0;
        for (int k = 0; k < q->n; k++) lv += i >= q->thr[k];
        return lv;
    }
    return -quant_q(q, i == 128 ? 127 : 256 - i);  /* read_quant_table mirrors 128 from 127 */
}
/* the 8-bit / 10-bit encoder's first quantiser level of d & 0xFF */
int ffv1o_quant_bits(int bits, int i) {
    const Quant q = oracle_quant(bits);
    return quant_q(&q, i);
}
int ffv1o_quant(int i /* 0..255 */) { return ffv1o_quant_bits(8, i); }

/* write_quant_table: run lengths of equal values over i = 0..127 */
static void write_quant_table(RC *c, int scale_is_zero, const Quant *q) {
    uint8_t st[CTX_SIZE];
    int last = 0, i;
    memset(st, 128, sizeof(st));
    for (i = 1; i < 128; i++)
        if (!scale_is_zero && quant_q(q, i) != quant_q(q, i - 1)) {
            put_symbol(c, st, i - last - 1, 0);
            last = i;
        }
    put_symbol(c, st, i - last - 1, 0);
}

/* Configuration record (extradata); returns its size (CRC parity included). */
int64_t ffv1o_extradata(int bits, int hsub, int vsub, int nh, int nv, uint8_t *out, int64_t cap) {
    RC c;
    uint8_t st[CTX_SIZE];
    int i;
    if (cap < 64) return -1;
    rc_init(&c, out, cap - 4);
    build_states(&c);
    memset(st, 128, sizeof(st));
    put_symbol(&c, st, 3, 0);      /* version */
    put_symbol(&c, st, 4, 0);      /* micro_version */
    put_symbol(&c, st, 1, 0);      /* coder_type: range coder, default table */
    put_symbol(&c, st, 0, 0);      /* colorspace: YCbCr */
    put_symbol(&c, st, bits, 0);   /* bits_per_raw_sample */
    put_rac(&c, st, 1);            /* chroma_planes */
    put_symbol(&c, st, hsub, 0);
    put_symbol(&c, st, vsub, 0);
    put_rac(&c, st, 0);            /* extra_plane (alpha) */
    put_symbol(&c, st, nh - 1, 0);
    put_symbol(&c, st, nv - 1, 0);
    put_symbol(&c, st, 1, 0);      /* quant_table_set_count */
    const Quant q = oracle_quant(bits);
    for (i = 0; i < 5; i++) write_quant_table(&c, i >= 3, &q);
    put_rac(&c, st, 0);            /* states_coded[0] */
    put_symbol(&c, st, 1, 0);      /* ec: slice CRCs */
    put_symbol(&c, st, 1, 0);      /* intra: every frame a keyframe */
    /* A 0 bit at state 129 before the flush, as every slice ends (ffv1enc.c
     * encode_frame): rc_terminate leaves the last byte to whatever follows
     * (here the CRC), and only a decoded value inside the interval BEFORE that
     * bit is guaranteed -- the reader never reads the bit itself. */
    uint8_t s129 = 129;
    put_rac(&c, &s129, 0);
    int64_t n = rc_terminate(&c);
    if (c.overflow) return -1;
    put_be32(out + n, ffv1o_crc(0, out, n));
    return n + 4;
}

/* ---- samples and context (encode_plane / encode_line) ------------------- */
static inline int median3(int a, int b, int c) {
    if (a > b) { int t = a; a = b; b = t; }
    return c < a ? a : (c > b ? b : c);
}

/* sample (x, y) of a slice plane with the encoder's border rules:
 * above the slice top -> 0; left of column 0 -> the sample above it;
 * right of the last column -> the sample to its left (top row only). */
typedef struct {
    const uint8_t *base;
    int64_t ls;
    int bytes, w, h;
} Plane;

static inline int px(const Plane *p, int x, int y) {
    if (y < 0) return 0;
    const uint8_t *r = p->base + (int64_t)y * p->ls;
    return p->bytes == 2 ? ((const uint16_t *)r)[x] : r[x];
}

static inline void neighbours(const Plane *p, int x, int y, int *L, int *TL, int *T, int *TR) {
    *T = px(p, x, y - 1);
    *L = x > 0 ? px(p, x - 1, y) : *T;
    *TL = x > 0 ? px(p, x - 1, y - 1) : px(p, 0, y - 2);
    *TR = x + 1 < p->w ? px(p, x + 1, y - 1) : *T;
}

static inline int fold(int diff, int bits) {
    const int m = 1 << bits;
    diff &= m - 1;
    return diff >= (m >> 1) ? diff - m : diff;
}

static void encode_plane(RC *c, uint8_t (*st)[CTX_SIZE], const Plane *p, int bits) {
    const Quant q = oracle_quant(bits);
    const int lv = levels(&q);
    for (int y = 0; y < p->h; y++)
        for (int x = 0; x < p->w; x++) {
            int L, TL, T, TR;
            neighbours(p, x, y, &L, &TL, &T, &TR);
            int ctx = quant_q(&q, (L - TL) & 0xFF) + lv * (quant_q(&q, (TL - T) & 0xFF) +
                      lv * quant_q(&q, (T - TR) & 0xFF));
            int diff = px(p, x, y) - median3(L, L + T - TL, T);
            if (ctx < 0) { ctx = -ctx; diff = -diff; }
            put_symbol(c, st[ctx], fold(diff, bits), 1);
        }
}

/* One slice (sx, sy) of a frame; `first` codes the frame's keyframe bit.
 * Returns the coded size (before the footer), -1 on overflow. */
int64_t ffv1o_encode_slice(const uint8_t *const planes[3], const int64_t ls[3], int w, int h, int bits, int hsub,
                           int vsub, int nh, int nv, int sx, int sy, uint8_t *out, int64_t cap) {
    RC c;
    uint8_t st[CTX_SIZE];
    const int bytes = bits > 8 ? 2 : 1;
    const int x0 = (int)((int64_t)sx * w / nh), x1 = (int)((int64_t)(sx + 1) * w / nh);
    const int y0 = (int)((int64_t)sy * h / nv), y1 = (int)((int64_t)(sy + 1) * h / nv);
    uint8_t (*states)[NCTX][CTX_SIZE] = malloc(sizeof(uint8_t[2][NCTX][CTX_SIZE]));
    if (!states) return -1;
    memset(states, 128, sizeof(uint8_t[2][NCTX][CTX_SIZE]));
    rc_init(&c, out, cap);
    build_states(&c);
    if (sx == 0 && sy == 0) {
        uint8_t key = 128;
        put_rac(&c, &key, 1);
    }
    memset(st, 128, sizeof(st));
    put_symbol(&c, st, sx, 0);
    put_symbol(&c, st, sy, 0);
    put_symbol(&c, st, 0, 0);  /* slice width - 1 in slice units */
    put_symbol(&c, st, 0, 0);
    put_symbol(&c, st, 0, 0);  /* quant_table_set_index, luma */
    put_symbol(&c, st, 0, 0);  /* chroma */
    put_symbol(&c, st, 3, 0);  /* picture_structure: progressive */
    put_symbol(&c, st, 1, 0);  /* sample aspect ratio 1:1 (setsar=1/1) */
    put_symbol(&c, st, 1, 0);
    for (int p = 0; p < 3; p++) {
        const int cs = p ? 1 : 0;
        const int px0 = p ? x0 >> hsub : x0, py0 = p ? y0 >> vsub : y0;
        Plane pl;
        pl.bytes = bytes;
        pl.ls = ls[p];
        pl.w = p ? ((x1 - x0) + (1 << hsub) - 1) >> hsub : x1 - x0;
        pl.h = p ? ((y1 - y0) + (1 << vsub) - 1) >> vsub : y1 - y0;
        pl.base = planes[p] + (int64_t)py0 * ls[p] + (int64_t)px0 * bytes;
        encode_plane(&c, states[cs], &pl, bits);
    }
    uint8_t s129 = 129;
    put_rac(&c, &s129, 0);
    int64_t n = rc_terminate(&c);
    free(states);
    return c.overflow ? -1 : n;
}

/* Slice footer: 24-bit size, error status 0, CRC-32 parity over the slice. */
int64_t ffv1o_slice_footer(uint8_t *slice, int64_t n) {
    slice[n] = (uint8_t)(n >> 16); slice[n + 1] = (uint8_t)(n >> 8); slice[n + 2] = (uint8_t)n;
    slice[n + 3] = 0;
    put_be32(slice + n + 4, ffv1o_crc(0, slice, n + 4));
    return n + 8;
}

/* A whole frame packet: slices in raster order, each followed by its footer. */
int64_t ffv1o_encode_frame(const uint8_t *const planes[3], const int64_t ls[3], int w, int h, int bits, int hsub,
                           int vsub, int nh, int nv, uint8_t *out, int64_t cap) {
    int64_t off = 0;
    for (int sy = 0; sy < nv; sy++)
        for (int sx = 0; sx < nh; sx++) {
            if (cap - off < 16) return -1;
            int64_t n = ffv1o_encode_slice(planes, ls, w, h, bits, hsub, vsub, nh, nv, sx, sy, out + off,
                                           cap - off - 8);
            if (n < 0) return -1;
            off += ffv1o_slice_footer(out + off, n);
        }
    return off;
}

/* ---- decoder (ffv1dec.c semantics, for the round trip) ------------------ */
typedef struct {
    int version, micro, coder, colorspace, bits, chroma, hsub, vsub, alpha, nh, nv, ntables, ec, intra;
    int ctx_count;
    int16_t q[5][256];
} Cfg;

static int read_quant_table(RD *d, int16_t *t, int scale) {
    uint8_t st[CTX_SIZE];
    int v, i = 0;
    memset(st, 128, sizeof(st));
    for (v = 0; i < 128; v++) {
        unsigned len = (unsigned)get_symbol(d, st, 0) + 1u;
        if (len > (unsigned)(128 - i) || !len) return -1;
        while (len--) t[i++] = (int16_t)(scale * v);
    }
    for (i = 1; i < 128; i++) t[256 - i] = (int16_t)-t[i];
    t[128] = (int16_t)-t[127];
    return 2 * v - 1;
}

/* Parse and check a configuration record; fills 16 ints of `info`:
 * version, micro, coder, colorspace, bits, chroma, hsub, vsub, alpha, nh, nv,
 * tables, ec, intra, context count, crc_ok. Returns 0 or -1. */
static int parse_cfg(const uint8_t *x, int64_t n, Cfg *f, int *crc_ok) {
    RD d;
    uint8_t st[CTX_SIZE];
    memset(f, 0, sizeof(*f));
    *crc_ok = n >= 4 && ffv1o_crc(0, x, n) == 0;
    rd_init(&d, x, n);
    memset(st, 128, sizeof(st));
    f->version = get_symbol(&d, st, 0);
    if (f->version != 3) return -1;
    f->micro = get_symbol(&d, st, 0);
    f->coder = get_symbol(&d, st, 0);
    if (f->coder != 1) return -1;
    f->colorspace = get_symbol(&d, st, 0);
    f->bits = get_symbol(&d, st, 0);
    f->chroma = get_rac(&d, st);
    f->hsub = get_symbol(&d, st, 0);
    f->vsub = get_symbol(&d, st, 0);
    f->alpha = get_rac(&d, st);
    f->nh = get_symbol(&d, st, 0) + 1;
    f->nv = get_symbol(&d, st, 0) + 1;
    f->ntables = get_symbol(&d, st, 0);
    if (f->ntables != 1) return -1;
    int cc = 1;
    for (int i = 0; i < 5; i++) {
        int r = read_quant_table(&d, f->q[i], cc);
        if (r < 0) return -1;
        cc *= r;
    }
    f->ctx_count = (cc + 1) / 2;
    if (get_rac(&d, st)) return -1;  /* initial states: not produced here */
    f->ec = get_symbol(&d, st, 0);
    f->intra = get_symbol(&d, st, 0);
    return 0;
}

int ffv1o_parse_extradata(const uint8_t *x, int64_t n, int *info) {
    Cfg f;
    int ok;
    int r = parse_cfg(x, n, &f, &ok);
    const int v[16] = {f.version, f.micro, f.coder, f.colorspace, f.bits, f.chroma, f.hsub, f.vsub, f.alpha,
                       f.nh, f.nv, f.ntables, f.ec, f.intra, f.ctx_count, ok};
    memcpy(info, v, sizeof(v));
    return r;
}

static void decode_plane(RD *d, uint8_t (*st)[CTX_SIZE], const Cfg *f, uint8_t *base, int64_t ls, int w, int h,
                         int bytes) {
    Plane p;
    p.base = base; p.ls = ls; p.bytes = bytes; p.w = w; p.h = h;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            int L, TL, T, TR;
            neighbours(&p, x, y, &L, &TL, &T, &TR);
            int ctx = f->q[0][(L - TL) & 0xFF] + f->q[1][(TL - T) & 0xFF] + f->q[2][(T - TR) & 0xFF];
            int sign = 0;
            if (ctx < 0) { ctx = -ctx; sign = 1; }
            int diff = get_symbol(d, st[ctx], 1);
            if (sign) diff = -diff;
            int v = (median3(L, L + T - TL, T) + diff) & ((1 << f->bits) - 1);
            uint8_t *r = base + (int64_t)y * ls;
            if (bytes == 2) ((uint16_t *)r)[x] = (uint16_t)v;
            else r[x] = (uint8_t)v;
        }
}

/* Decode a frame packet into caller planes (w x h, linesizes ls).  Returns 0,
 * or a negative code: -1 bad record, -2 slice chain / size, -3 slice CRC,
 * -4 slice header, -5 bytestream end mismatch (FFmpeg's check). */
int ffv1o_decode_frame(const uint8_t *extra, int64_t extra_n, const uint8_t *pkt, int64_t n, int w, int h,
                       uint8_t *const planes[3], const int64_t ls[3]) {
    Cfg f;
    int ok;
    if (parse_cfg(extra, extra_n, &f, &ok) || !ok) return -1;
    const int ns = f.nh * f.nv, trailer = 3 + 5 * (f.ec != 0);
    const int bytes = f.bits > 8 ? 2 : 1;
    int64_t *start = malloc(sizeof(int64_t) * ns), *len = malloc(sizeof(int64_t) * ns);
    int64_t end = n;
    int rc = 0;
    for (int i = ns - 1; i >= 0; i--) {
        if (end < trailer) { rc = -2; goto out; }
        int64_t v = ((int64_t)pkt[end - trailer] << 16 | pkt[end - trailer + 1] << 8 | pkt[end - trailer + 2]) + trailer;
        if (v > end) { rc = -2; goto out; }
        end -= v;
        if (f.ec && ffv1o_crc(0, pkt + end, v) != 0) { rc = -3; goto out; }
        start[i] = end;
        len[i] = v;
    }
    for (int i = 0; i < ns; i++) {
        RD d;
        uint8_t st[CTX_SIZE];
        rd_init(&d, pkt + start[i], len[i]);
        if (i == 0) {
            uint8_t key = 128;
            if (!get_rac(&d, &key)) { rc = -4; goto out; }
        }
        memset(st, 128, sizeof(st));
        int sx = get_symbol(&d, st, 0), sy = get_symbol(&d, st, 0);
        int sw = get_symbol(&d, st, 0) + 1, sh = get_symbol(&d, st, 0) + 1;
        int q0 = get_symbol(&d, st, 0), q1 = get_symbol(&d, st, 0);
        int ps = get_symbol(&d, st, 0), sn = get_symbol(&d, st, 0), sd = get_symbol(&d, st, 0);
        (void)sn; (void)sd;
        if (sx < 0 || sy < 0 || sx > f.nh - sw || sy > f.nv - sh || q0 || q1 || ps != 3) { rc = -4; goto out; }
        const int x0 = (int)((int64_t)sx * w / f.nh), x1 = (int)((int64_t)(sx + sw) * w / f.nh);
        const int y0 = (int)((int64_t)sy * h / f.nv), y1 = (int)((int64_t)(sy + sh) * h / f.nv);
        uint8_t (*states)[NCTX][CTX_SIZE] = malloc(sizeof(uint8_t[2][NCTX][CTX_SIZE]));
        memset(states, 128, sizeof(uint8_t[2][NCTX][CTX_SIZE]));
        for (int p = 0; p < 3; p++) {
            const int cw = p ? ((x1 - x0) + (1 << f.hsub) - 1) >> f.hsub : x1 - x0;
            const int ch = p ? ((y1 - y0) + (1 << f.vsub) - 1) >> f.vsub : y1 - y0;
            const int px0 = p ? x0 >> f.hsub : x0, py0 = p ? y0 >> f.vsub : y0;
            decode_plane(&d, states[p ? 1 : 0], &f, planes[p] + (int64_t)py0 * ls[p] + (int64_t)px0 * bytes, ls[p],
                         cw, ch, bytes);
        }
        free(states);
        uint8_t s129 = 129;
        get_rac(&d, &s129);
        if ((d.end - d.p) - 2 - 5 * (f.ec != 0) != 0) { rc = -5; goto out; }
    }
out:
    free(start);
    free(len);
    return rc;
}

/* ========================================================================
 * General FFV1 version 3 streams -- what `ffmpeg -c:v ffv1 -level 3 -coder 1
 * -context 1 -slicecrc 1` writes (/root/reference/lib/ffmpeg.py:993, :1047)
 * and pixpath's intra subset above does not:
 *   - a transmitted state-transition table (coder_type 2, AC_RANGE_CUSTOM_TAB:
 *     ffv1enc.c write_extradata writes state_transition[i] - one_state[i] as
 *     signed symbols for i = 1..255; ffv1.c ff_ffv1_init_slice_state installs
 *     it as one_state / zero_state[256 - i] = 256 - one_state[i] of every slice
 *     coder, so everything after the keyframe bit uses it);
 *   - several quantisation table sets (quant_table_count <= 8) of up to 5
 *     inputs -- get_context (ffv1_template.c) adds q[3][(LL - L) & 0xFF] and
 *     q[4][(TT - T) & 0xFF] when q[3][127] or q[4][127] is non-zero -- with the
 *     set per plane chosen in each slice header (quant_table_index);
 *   - initial context states per table set (states_coded, delta-coded over
 *     the previous context with 32 separate state arrays);
 *   - inter frames (intra = 0): a slice's context states carry over from the
 *     same slice of the previous frame until the next keyframe (FFmpeg's
 *     default GOP of 12); ff_ffv1_clear_slice_state resets them to the
 *     initial states on a keyframe.
 * Border samples follow FFmpeg's sample buffers exactly (ffv1enc.c
 * encode_plane: a ring of 3 rows of w + 6 int16 with 3 before each row;
 * ffv1dec.c decode_plane: 2 rows, the current one overwriting the row two
 * above in place): above the slice -> 0; L at x = 0 -> T; LT at x = 0 -> the
 * row two above's first sample; RT at x = w - 1 -> T; LL at x = 0 -> 0, at
 * x = 1 -> T(0); TT -> the row two above (0 for the first two rows).
 * The configuration record ends with ff_rac_terminate(c, 0) (no state-129 bit).
 * The quantisation tables FFmpeg uses (quant11 / quant5 / quant9_10bit /
 * quant5_10bit) are data in the record; the tests build tables of the same
 * shape.  PARITY UNPINNED against FFmpeg (absent here), like the rest.
 * ====================================================================== */
#define GEN_MAX_TABLES 8
#define GEN_MAX_CTX 16384  /* (32768 + 1) / 2: read_quant_tables' bound */

typedef struct {
    int bits, hsub, vsub, nh, nv, micro, coder, ntables, ec, intra, gop, tidx[2];
    uint8_t trans[256];                       /* coder 2: state_transition[1..255] */
    uint8_t levels[GEN_MAX_TABLES][5][128];   /* unscaled quantiser level of d = 0..127 */
    uint8_t has_init[GEN_MAX_TABLES];
    const uint8_t *init[GEN_MAX_TABLES];      /* [context_count][32] where has_init */
} ffv1o_prof;

/* scaled tables of one set (write_quant_tables' input / read_quant_tables' output) */
static int gen_tables(const uint8_t lv[5][128], int16_t q[5][256]) {
    int cc = 1;
    for (int t = 0; t < 5; t++) {
        int v = 0;
        for (int i = 0; i < 128; i++) {
            if (i && lv[t][i] != lv[t][i - 1]) {
                if (lv[t][i] != lv[t][i - 1] + 1) return -1;  /* levels step by one (run lengths) */
                v++;
            }
            q[t][i] = (int16_t)(cc * lv[t][i]);
        }
        if (lv[t][0]) return -1;
        for (int i = 1; i < 128; i++) q[t][256 - i] = (int16_t)-q[t][i];
        q[t][128] = (int16_t)-q[t][127];
        cc *= 2 * (v + 1) - 1;
        if (cc > 32768) return -1;
    }
    return (cc + 1) / 2;
}

static void gen_write_table(RC *c, const uint8_t *lv) {
    uint8_t st[CTX_SIZE];
    int last = 0, i;
    memset(st, 128, sizeof(st));
    for (i = 1; i < 128; i++)
        if (lv[i] != lv[i - 1]) {
            put_symbol(c, st, i - last - 1, 0);
            last = i;
        }
    put_symbol(c, st, i - last - 1, 0);
}

static void gen_custom_states(RC *c, const ffv1o_prof *pf) {
    if (pf->coder != 2) return;
    for (int i = 1; i < 256; i++) {
        c->one_state[i] = pf->trans[i];
        c->zero_state[256 - i] = (uint8_t)(256 - c->one_state[i]);
    }
}

int64_t ffv1o_gen_extradata(const ffv1o_prof *pf, uint8_t *out, int64_t cap) {
    RC c;
    uint8_t st[CTX_SIZE], st2[CTX_SIZE][CTX_SIZE];
    int16_t q[5][256];
    if (cap < 64 || pf->ntables < 1 || pf->ntables > GEN_MAX_TABLES) return -1;
    rc_init(&c, out, cap - 4);
    build_states(&c);
    memset(st, 128, sizeof(st));
    memset(st2, 128, sizeof(st2));
    put_symbol(&c, st, 3, 0);
    put_symbol(&c, st, pf->micro, 0);
    put_symbol(&c, st, pf->coder, 0);
    if (pf->coder == 2)
        for (int i = 1; i < 256; i++) put_symbol(&c, st, pf->trans[i] - c.one_state[i], 1);
    put_symbol(&c, st, 0, 0);
    put_symbol(&c, st, pf->bits, 0);
    put_rac(&c, st, 1);
    put_symbol(&c, st, pf->hsub, 0);
    put_symbol(&c, st, pf->vsub, 0);
    put_rac(&c, st, 0);
    put_symbol(&c, st, pf->nh - 1, 0);
    put_symbol(&c, st, pf->nv - 1, 0);
    put_symbol(&c, st, pf->ntables, 0);
    for (int i = 0; i < pf->ntables; i++)
        for (int t = 0; t < 5; t++) gen_write_table(&c, pf->levels[i][t]);
    for (int i = 0; i < pf->ntables; i++) {
        const int cc = gen_tables(pf->levels[i], q);
        if (cc < 0) return -1;
        if (!pf->has_init[i]) {
            put_rac(&c, st, 0);
            continue;
        }
        put_rac(&c, st, 1);
        for (int j = 0; j < cc; j++)
            for (int k = 0; k < CTX_SIZE; k++) {
                const int pred = j ? pf->init[i][(j - 1) * CTX_SIZE + k] : 128;
                put_symbol(&c, st2[k], (int8_t)(pf->init[i][j * CTX_SIZE + k] - pred), 1);
            }
    }
    put_symbol(&c, st, pf->ec, 0);
    if (pf->micro > 2) put_symbol(&c, st, pf->intra, 0);
    int64_t n = rc_terminate(&c);
    if (c.overflow) return -1;
    put_be32(out + n, ffv1o_crc(0, out, n));
    return n + 4;
}

static int gen_context(const int16_t (*q)[256], int five, const int16_t *src, const int16_t *last, const int16_t *last2) {
    const int LT = last[-1], T = last[0], RT = last[1], L = src[-1];
    int ctx = q[0][(L - LT) & 0xFF] + q[1][(LT - T) & 0xFF] + q[2][(T - RT) & 0xFF];
    if (five) ctx += q[3][(src[-2] - L) & 0xFF] + q[4][(last2[0] - T) & 0xFF];
    return ctx;
}

/* encode_plane / encode_line (ffv1enc.c) on the 3-row ring */
static void gen_encode_plane(RC *c, uint8_t (*st)[CTX_SIZE], const int16_t (*q)[256], const Plane *p, int bits,
                             int16_t *buf) {
    const int w = p->w, h = p->h, five = q[3][127] || q[4][127];
    int16_t *s[3];
    memset(buf, 0, sizeof(int16_t) * 3 * (w + 6));
    for (int y = 0; y < h; y++) {
        for (int i = 0; i < 3; i++) s[i] = buf + (w + 6) * ((h + i - y) % 3) + 3;
        s[0][-1] = s[1][0];
        s[1][w] = s[1][w - 1];
        for (int x = 0; x < w; x++) s[0][x] = (int16_t)px(p, x, y);
        for (int x = 0; x < w; x++) {
            int ctx = gen_context(q, five, s[0] + x, s[1] + x, s[2] + x);
            int diff = s[0][x] - median3(s[0][x - 1], s[0][x - 1] + s[1][x] - s[1][x - 1], s[1][x]);
            if (ctx < 0) { ctx = -ctx; diff = -diff; }
            put_symbol(c, st[ctx], fold(diff, bits), 1);
        }
    }
}

typedef struct {
    ffv1o_prof pf;
    int w, h, frame;
    int16_t q[GEN_MAX_TABLES][5][256];
    int cc[GEN_MAX_TABLES];
    uint8_t *states;  /* [nh * nv][2][GEN_MAX_CTX][32]: slice, plane set */
    int16_t *buf;
} ffv1o_gen_enc;

static void gen_clear(uint8_t *st, const ffv1o_prof *pf, const int *cc, int ti) {
    if (pf->has_init[ti]) memcpy(st, pf->init[ti], (size_t)cc[ti] * CTX_SIZE);
    else memset(st, 128, (size_t)cc[ti] * CTX_SIZE);
}

void ffv1o_gen_encoder_destroy(ffv1o_gen_enc *e) {
    if (!e) return;
    free(e->states);
    free(e->buf);
    free(e);
}

ffv1o_gen_enc *ffv1o_gen_encoder_create(const ffv1o_prof *pf, int w, int h) {
    if (pf->ntables < 1 || pf->ntables > GEN_MAX_TABLES || pf->nh < 1 || pf->nv < 1 || pf->nh * pf->nv > 1024 ||
        pf->tidx[0] < 0 || pf->tidx[0] >= pf->ntables || pf->tidx[1] < 0 || pf->tidx[1] >= pf->ntables ||
        (pf->coder != 1 && pf->coder != 2) || pf->gop < 1)
        return NULL;
    ffv1o_gen_enc *e = calloc(1, sizeof(*e));
    if (!e) return NULL;
    e->pf = *pf;
    e->w = w;
    e->h = h;
    for (int i = 0; i < pf->ntables; i++)
        if ((e->cc[i] = gen_tables(pf->levels[i], e->q[i])) < 0) {
            free(e);
            return NULL;
        }
    e->states = malloc((size_t)pf->nh * pf->nv * 2 * GEN_MAX_CTX * CTX_SIZE);
    e->buf = malloc(sizeof(int16_t) * 3 * (w + 6));
    if (!e->states || !e->buf) {
        ffv1o_gen_encoder_destroy(e);
        return NULL;
    }
    return e;
}

/* The next frame of the sequence (a keyframe every pf->gop frames): slices in
 * raster order with their footers.  Returns the packet size, -1 on overflow. */
int64_t ffv1o_gen_encode_frame(ffv1o_gen_enc *e, const uint8_t *const planes[3], const int64_t ls[3], uint8_t *out,
                               int64_t cap) {
    const ffv1o_prof *pf = &e->pf;
    const int key = e->frame % pf->gop == 0, bytes = pf->bits > 8 ? 2 : 1;
    int64_t off = 0;
    for (int si = 0; si < pf->nh * pf->nv; si++) {
        const int sx = si % pf->nh, sy = si / pf->nh;
        uint8_t *sst = e->states + (size_t)si * 2 * GEN_MAX_CTX * CTX_SIZE;
        if (cap - off < 16) return -1;
        RC c;
        uint8_t st[CTX_SIZE];
        rc_init(&c, out + off, cap - off - 8);
        build_states(&c);
        if (si == 0) {  /* the keyframe bit: frame coder, default table (encode_frame) */
            uint8_t ks = 128;
            put_rac(&c, &ks, key);
        }
        gen_custom_states(&c, pf);
        if (key) {
            gen_clear(sst, pf, e->cc, pf->tidx[0]);
            gen_clear(sst + (size_t)GEN_MAX_CTX * CTX_SIZE, pf, e->cc, pf->tidx[1]);
        }
        memset(st, 128, sizeof(st));  /* encode_slice_header */
        put_symbol(&c, st, sx, 0);
        put_symbol(&c, st, sy, 0);
        put_symbol(&c, st, 0, 0);
        put_symbol(&c, st, 0, 0);
        put_symbol(&c, st, pf->tidx[0], 0);
        put_symbol(&c, st, pf->tidx[1], 0);
        put_symbol(&c, st, 3, 0);
        put_symbol(&c, st, 1, 0);
        put_symbol(&c, st, 1, 0);
        const int x0 = (int)((int64_t)sx * e->w / pf->nh), x1 = (int)((int64_t)(sx + 1) * e->w / pf->nh);
        const int y0 = (int)((int64_t)sy * e->h / pf->nv), y1 = (int)((int64_t)(sy + 1) * e->h / pf->nv);
        for (int p = 0; p < 3; p++) {
            const int cs = p ? 1 : 0;
            Plane pl;
            pl.bytes = bytes;
            pl.ls = ls[p];
            pl.w = p ? ((x1 - x0) + (1 << pf->hsub) - 1) >> pf->hsub : x1 - x0;
            pl.h = p ? ((y1 - y0) + (1 << pf->vsub) - 1) >> pf->vsub : y1 - y0;
            const int px0 = p ? x0 >> pf->hsub : x0, py0 = p ? y0 >> pf->vsub : y0;
            pl.base = planes[p] + (int64_t)py0 * ls[p] + (int64_t)px0 * bytes;
            gen_encode_plane(&c, (uint8_t (*)[CTX_SIZE])(sst + (size_t)cs * GEN_MAX_CTX * CTX_SIZE),
                             (const int16_t (*)[256])e->q[pf->tidx[cs]], &pl, pf->bits, e->buf);
        }
        uint8_t s129 = 129;
        put_rac(&c, &s129, 0);
        int64_t n = rc_terminate(&c);
        if (c.overflow) return -1;
        off += ffv1o_slice_footer(out + off, n);
    }
    e->frame++;
    return off;
}

/* ---- general decoder (ffv1dec.c read_extra_header / decode_frame /
 * decode_slice_header / decode_plane / decode_line) -------------------- */
typedef struct {
    int w, h, bits, hsub, vsub, nh, nv, micro, coder, ntables, ec, intra;
    uint8_t trans[256];
    int16_t q[GEN_MAX_TABLES][5][256];
    int cc[GEN_MAX_TABLES];
    uint8_t *init[GEN_MAX_TABLES];    /* [cc][32]: 128s unless transmitted */
    uint8_t *states;                  /* [slices][2][GEN_MAX_CTX][32] */
    int *sidx;                        /* [slices][2]: the table set each plane's states follow */
    int key_ok;
    int16_t *buf;
} ffv1o_gen_dec;

void ffv1o_gen_decoder_destroy(ffv1o_gen_dec *d) {
    if (!d) return;
    for (int i = 0; i < GEN_MAX_TABLES; i++) free(d->init[i]);
    free(d->states);
    free(d->sidx);
    free(d->buf);
    free(d);
}

/* info (16 ints): version, micro, coder, bits, hsub, vsub, nh, nv, tables,
 * ec, intra, context count of sets 0 / 1, initial states of sets 0 / 1, crc ok */
ffv1o_gen_dec *ffv1o_gen_decoder_create(const uint8_t *x, int64_t n, int w, int h, int *info) {
    RD r;
    uint8_t st[CTX_SIZE], st2[CTX_SIZE][CTX_SIZE];
    int crc_ok = n >= 4 && ffv1o_crc(0, x, n) == 0;
    memset(info, 0, 16 * sizeof(int));
    info[15] = crc_ok;
    if (n < 8) return NULL;
    ffv1o_gen_dec *d = calloc(1, sizeof(*d));
    if (!d) return NULL;
    d->w = w;
    d->h = h;
    rd_init(&r, x, n - 4);  /* read_extra_header: bytestream_end -= 4 */
    memset(st, 128, sizeof(st));
    memset(st2, 128, sizeof(st2));
    const int version = get_symbol(&r, st, 0);
    d->micro = get_symbol(&r, st, 0);
    d->coder = get_symbol(&r, st, 0);
    info[0] = version; info[1] = d->micro; info[2] = d->coder;
    if (version != 3 || (d->coder != 1 && d->coder != 2)) goto bad;
    if (d->coder == 2)
        for (int i = 1; i < 256; i++) {
            const int v = get_symbol(&r, st, 1) + r.one_state[i];
            if (v < 1 || v > 255) goto bad;
            d->trans[i] = (uint8_t)v;
        }
    if (get_symbol(&r, st, 0) != 0) goto bad;  /* colorspace YCbCr */
    d->bits = get_symbol(&r, st, 0);
    if (!get_rac(&r, st)) goto bad;            /* chroma_planes */
    d->hsub = get_symbol(&r, st, 0);
    d->vsub = get_symbol(&r, st, 0);
    if (get_rac(&r, st)) goto bad;             /* transparency */
    d->nh = get_symbol(&r, st, 0) + 1;
    d->nv = get_symbol(&r, st, 0) + 1;
    d->ntables = get_symbol(&r, st, 0);
    info[3] = d->bits; info[4] = d->hsub; info[5] = d->vsub; info[6] = d->nh; info[7] = d->nv; info[8] = d->ntables;
    if (d->bits < 8 || d->bits > 10 || d->hsub > 1 || d->vsub > 1 || d->nh < 1 || d->nv < 1 || d->nh > w ||
        d->nv > h || d->nh * d->nv > 1024 || d->ntables < 1 || d->ntables > GEN_MAX_TABLES)
        goto bad;
    for (int i = 0; i < d->ntables; i++) {
        int cc = 1;
        for (int t = 0; t < 5; t++) {
            const int lv = read_quant_table(&r, d->q[i][t], cc);
            if (lv < 0) goto bad;
            cc *= lv;
            if (cc > 32768) goto bad;
        }
        d->cc[i] = (cc + 1) / 2;
    }
    for (int i = 0; i < d->ntables; i++) {
        d->init[i] = malloc((size_t)d->cc[i] * CTX_SIZE);
        if (!d->init[i]) goto bad;
        memset(d->init[i], 128, (size_t)d->cc[i] * CTX_SIZE);
        if (get_rac(&r, st)) {
            if (i < 2) info[13 + i] = 1;
            for (int j = 0; j < d->cc[i]; j++)
                for (int k = 0; k < CTX_SIZE; k++) {
                    const int pred = j ? d->init[i][(j - 1) * CTX_SIZE + k] : 128;
                    d->init[i][j * CTX_SIZE + k] = (uint8_t)((pred + get_symbol(&r, st2[k], 1)) & 0xFF);
                }
        }
    }
    d->ec = get_symbol(&r, st, 0);
    d->intra = d->micro > 2 ? get_symbol(&r, st, 0) : 0;
    info[9] = d->ec; info[10] = d->intra; info[11] = d->cc[0]; info[12] = d->ntables > 1 ? d->cc[1] : 0;
    if (!crc_ok || d->ec < 0 || d->ec > 1) goto bad;
    d->states = malloc((size_t)d->nh * d->nv * 2 * GEN_MAX_CTX * CTX_SIZE);
    d->sidx = calloc((size_t)d->nh * d->nv * 2, sizeof(int));
    d->buf = malloc(sizeof(int16_t) * 2 * (w + 6));
    if (!d->states || !d->sidx || !d->buf) goto bad;
    return d;
bad:
    ffv1o_gen_decoder_destroy(d);
    return NULL;
}

static void gen_decode_plane(RD *r, uint8_t (*st)[CTX_SIZE], const int16_t (*q)[256], uint8_t *base, int64_t ls,
                             int w, int h, int bits, int16_t *buf) {
    const int five = q[3][127] || q[4][127], bytes = bits > 8 ? 2 : 1;
    int16_t *s[2] = {buf + 3, buf + w + 6 + 3};
    memset(buf, 0, sizeof(int16_t) * 2 * (w + 6));
    for (int y = 0; y < h; y++) {
        int16_t *t = s[0];
        s[0] = s[1];
        s[1] = t;
        s[1][-1] = s[0][0];
        s[0][w] = s[0][w - 1];
        for (int x = 0; x < w; x++) {
            /* get_context(p, sample[1] + x, sample[0] + x, sample[1] + x): TT
             * is the row two above, still in the current row's buffer at x */
            int ctx = gen_context(q, five, s[1] + x, s[0] + x, s[1] + x);
            int sign = 0;
            if (ctx < 0) { ctx = -ctx; sign = 1; }
            int diff = get_symbol(r, st[ctx], 1);
            if (sign) diff = -diff;
            const int L = s[1][x - 1], T = s[0][x], LT = s[0][x - 1];
            s[1][x] = (int16_t)((median3(L, L + T - LT, T) + diff) & ((1 << bits) - 1));
        }
        uint8_t *row = base + (int64_t)y * ls;
        for (int x = 0; x < w; x++) {
            if (bytes == 2) ((uint16_t *)row)[x] = (uint16_t)s[1][x];
            else row[x] = (uint8_t)s[1][x];
        }
    }
}

/* Decode the next packet of the sequence (states carried from the previous
 * call's frame unless this one is a keyframe).  Returns 0, or -2 slice chain,
 * -3 slice CRC, -4 slice header, -5 bytestream end, -6 non-keyframe first. */
int ffv1o_gen_decode_frame(ffv1o_gen_dec *d, const uint8_t *pkt, int64_t n, uint8_t *const planes[3],
                           const int64_t ls[3], int *keyframe) {
    const int ns = d->nh * d->nv, trailer = 3 + 5 * (d->ec != 0), bytes = d->bits > 8 ? 2 : 1;
    int64_t start[1024], len[1024], end = n;
    for (int i = ns - 1; i >= 0; i--) {
        if (end < trailer) return -2;
        const int64_t v = ((int64_t)pkt[end - trailer] << 16 | pkt[end - trailer + 1] << 8 | pkt[end - trailer + 2]) +
                          trailer;
        if (i == 0 ? v != end : v > end) return -2;
        end -= v;
        if (d->ec && ffv1o_crc(0, pkt + end, v) != 0) return -3;
        start[i] = end;
        len[i] = v;
    }
    int key = 0;
    for (int i = 0; i < ns; i++) {
        RD r;
        uint8_t st[CTX_SIZE];
        rd_init(&r, pkt + start[i], len[i]);
        if (i == 0) {
            uint8_t ks = 128;
            key = get_rac(&r, &ks);
            if (keyframe) *keyframe = key;
            if (!key && !d->key_ok) return -6;
            d->key_ok = 1;
        }
        if (d->coder == 2)
            for (int k = 1; k < 256; k++) {
                r.one_state[k] = d->trans[k];
                r.zero_state[256 - k] = (uint8_t)(256 - d->trans[k]);
            }
        memset(st, 128, sizeof(st));
        const int sx = get_symbol(&r, st, 0), sy = get_symbol(&r, st, 0);
        const int sw = get_symbol(&r, st, 0) + 1, sh = get_symbol(&r, st, 0) + 1;
        int ti[2];
        ti[0] = get_symbol(&r, st, 0);
        ti[1] = get_symbol(&r, st, 0);
        (void)get_symbol(&r, st, 0);  /* picture structure */
        (void)get_symbol(&r, st, 0);  /* sample aspect ratio */
        (void)get_symbol(&r, st, 0);
        if (sx < 0 || sy < 0 || sw < 1 || sh < 1 || sx > d->nh - sw || sy > d->nv - sh || ti[0] < 0 ||
            ti[0] >= d->ntables || ti[1] < 0 || ti[1] >= d->ntables)
            return -4;
        uint8_t *sst = d->states + (size_t)i * 2 * GEN_MAX_CTX * CTX_SIZE;
        if (key)
            for (int c = 0; c < 2; c++) {
                memcpy(sst + (size_t)c * GEN_MAX_CTX * CTX_SIZE, d->init[ti[c]], (size_t)d->cc[ti[c]] * CTX_SIZE);
                d->sidx[2 * i + c] = ti[c];
            }
        else if (ti[0] != d->sidx[2 * i] || ti[1] != d->sidx[2 * i + 1])
            return -4;  /* a table set change without a keyframe (FFmpeg: states reallocated, undefined) */
        const int x0 = (int)((int64_t)sx * d->w / d->nh), x1 = (int)((int64_t)(sx + sw) * d->w / d->nh);
        const int y0 = (int)((int64_t)sy * d->h / d->nv), y1 = (int)((int64_t)(sy + sh) * d->h / d->nv);
        for (int p = 0; p < 3; p++) {
            const int cs = p ? 1 : 0;
            const int cw = p ? ((x1 - x0) + (1 << d->hsub) - 1) >> d->hsub : x1 - x0;
            const int ch = p ? ((y1 - y0) + (1 << d->vsub) - 1) >> d->vsub : y1 - y0;
            const int px0 = p ? x0 >> d->hsub : x0, py0 = p ? y0 >> d->vsub : y0;
            gen_decode_plane(&r, (uint8_t (*)[CTX_SIZE])(sst + (size_t)cs * GEN_MAX_CTX * CTX_SIZE),
                             (const int16_t (*)[256])d->q[ti[cs]],
                             planes[p] + (int64_t)py0 * ls[p] + (int64_t)px0 * bytes, ls[p], cw, ch, d->bits, d->buf);
        }
        uint8_t s129 = 129;
        get_rac(&r, &s129);
        if ((r.end - r.p) - 2 - 5 * (d->ec != 0) != 0) return -5;
    }
    return 0;
}
