// Host side of the FFV1 codec: state tables, CRC, configuration record, slice
// footers (see ffv1host.hpp).  The algorithms follow FFmpeg's ffv1enc.c /
// ffv1dec.c / rangecoder.c as published (RFC 9043); no HIP here.
#include "ffv1host.hpp"

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "../../include/pixpath.h"

namespace pp {

namespace {

int fail(std::string *err, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (err) *err = buf;
    return code;
}

// range encoder of the configuration record (rangecoder.c put_rac /
// renorm_encoder, ffv1enc.c put_symbol)
struct HostRC {
    int low = 0, range = 0xFF00, oc = 0, ob = -1;
    uint8_t zero[256], one[256];
    std::vector<uint8_t> out;
    HostRC() { rac_states(zero, one); }
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
    void terminate() {
        range = 0xFF;
        low += 0xFF;
        renorm();
        range = 0xFF;
        renorm();
    }
};

// range decoder (rangecoder.h get_rac / refill, ffv1dec.c get_symbol); reads
// never pass `end` (past it, refill shifts in zeros as FFmpeg's does)
struct HostRD {
    int low = 0, range = 0xFF00;
    const uint8_t *p = nullptr, *end = nullptr;
    uint8_t zero[256], one[256];
    HostRD(const uint8_t *b, int64_t n) {
        rac_states(zero, one);
        p = b;
        end = b + n;
        low = n >= 2 ? (b[0] << 8) | b[1] : 0;
        p = n >= 2 ? p + 2 : end;
        if (low >= 0xFF00) {
            low = 0xFF00;
            end = p;
        }
    }
    void refill() {
        if (range < 0x100) {
            range <<= 8;
            low <<= 8;
            if (p < end) low += *p++;
        }
    }
    int rac(uint8_t *st) {
        const int r1 = (range * *st) >> 8;
        range -= r1;
        if (low < range) {
            *st = zero[*st];
            refill();
            return 0;
        }
        low -= range;
        *st = one[*st];
        range = r1;
        refill();
        return 1;
    }
    int symbol(uint8_t *st) {  // unsigned; -1 past 31 exponent bits (corrupt)
        bool bad = false;
        const int v = ssymbol(st, false, &bad);
        return bad ? -1 : v;
    }
    // get_symbol (ffv1dec.c): sign at state 11 + min(e, 10); *bad past 30 exponent bits
    int ssymbol(uint8_t *st, bool is_signed, bool *bad) {
        if (rac(st)) return 0;
        int e = 0;
        while (rac(st + 1 + std::min(e, 9))) {
            if (++e > 30) {
                *bad = true;
                return 0;
            }
        }
        int a = 1;
        for (int i = e - 1; i >= 0; i--) a += a + rac(st + 22 + std::min(i, 9));
        return is_signed && rac(st + 11 + std::min(e, 10)) ? -a : a;
    }
};

}  // namespace

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

void crc_table(uint32_t t[256]) {
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i << 24;
        for (int j = 0; j < 8; j++) c = (c << 1) ^ ((c & 0x80000000u) ? 0x04C11DB7u : 0u);
        t[i] = c;
    }
}

int ffv1_quant(int i, const Ffv1Quant &q) {
    if (i >= 128) return -ffv1_quant(i == 128 ? 127 : 256 - i, q);
    int lv = 0;
    for (int k = 0; k < q.n; ++k) lv += i >= q.thr[k];
    return lv;
}

Ffv1Quant ffv1_default_quant(int depth) {
    // Small context sets keep the slices' adaptive states cache-resident on
    // the GPU: the coder and the decoder load one context's block per sample
    // (profiles/r5/ffv1_context_model.txt: 63 contexts encode and decode ~15 %
    // faster than 666 on the bench content, files 4 % smaller).  10 bits:
    // thresholds 4, 32 (5 levels, 63 contexts); 8 bits, whose differences are
    // 4x smaller, 1, 3, 8 (7 levels, 172 contexts: 5 levels cost 8-bit smooth
    // content ~15 % in file size)
    Ffv1Quant q;
    if (depth > 8) {
        q.n = 2; q.thr[0] = 4; q.thr[1] = 32;
    } else {
        q.n = 3; q.thr[0] = 1; q.thr[1] = 3; q.thr[2] = 8;
    }
    return q;
}

std::vector<uint8_t> ffv1_write_record(int depth, int hsub, int vsub, int slices_h, int slices_v,
                                       const Ffv1Quant &q) {
    HostRC c;
    uint8_t st[kFfv1CtxBytes];
    std::memset(st, 128, sizeof(st));
    const int v1[] = {3, 4, 1, 0, depth};  // version, micro_version, coder_type, colorspace, bits
    for (int v : v1) c.symbol(st, v);
    c.rac(st, 1);  // chroma_planes
    c.symbol(st, hsub);
    c.symbol(st, vsub);
    c.rac(st, 0);  // extra_plane
    c.symbol(st, slices_h - 1);
    c.symbol(st, slices_v - 1);
    c.symbol(st, 1);  // quant_table_set_count
    for (int t = 0; t < 5; t++) {
        uint8_t qs[kFfv1CtxBytes];
        std::memset(qs, 128, sizeof(qs));
        int last = 0, i;
        for (i = 1; i < 128; i++)
            if (t < 3 && ffv1_quant(i, q) != ffv1_quant(i - 1, q)) {
                c.symbol(qs, i - last - 1);
                last = i;
            }
        c.symbol(qs, i - last - 1);
    }
    c.rac(st, 0);     // states_coded
    c.symbol(st, 1);  // ec
    c.symbol(st, 1);  // intra
    uint8_t s129 = 129;
    c.rac(&s129, 0);
    c.terminate();
    uint32_t t[256];
    crc_table(t);
    uint32_t crc = 0;
    for (uint8_t b : c.out) crc = (crc << 8) ^ t[(crc >> 24) ^ b];
    std::vector<uint8_t> rec = c.out;
    for (int k = 3; k >= 0; k--) rec.push_back((uint8_t)(crc >> (8 * k)));
    return rec;
}

int ffv1_parse_record(const uint8_t *extra, int size, int w, int h, Ffv1Record *rec, std::string *err) {
    if (!extra || !rec) return fail(err, PP_ERR_INVALID, "null argument");
    if (size < 8) return fail(err, PP_ERR_INVALID, "configuration record of %d bytes", size);
    {
        uint32_t t[256];
        crc_table(t);
        uint32_t crc = 0;
        for (int i = 0; i < size; i++) crc = (crc << 8) ^ t[(crc >> 24) ^ extra[i]];
        if (crc) return fail(err, PP_ERR_INVALID, "configuration record CRC mismatch");
    }
    Ffv1Record R;
    HostRD r(extra, size - 4);  // read_extra_header: the CRC is not range-coded data
    uint8_t st[kFfv1CtxBytes];
    std::memset(st, 128, sizeof(st));
    bool bad = false;
    const int version = r.symbol(st);
    R.micro = r.symbol(st);
    R.coder = r.symbol(st);
    if (version != 3 || R.micro < 0 || (R.coder != 1 && R.coder != 2))
        return fail(err, PP_ERR_UNSUPPORTED, "FFV1 record: version %d coder %d (supported: version 3, range coder 1 or 2)",
                    version, R.coder);
    rac_states(R.zero_state, R.one_state);
    if (R.coder == 2) {  // AC_RANGE_CUSTOM_TAB: state_transition[i] - one_state[i], signed
        uint8_t one[256];
        for (int i = 1; i < 256; i++) {
            const int v = r.ssymbol(st, true, &bad) + r.one[i];
            if (bad || v < 1 || v > 255) return fail(err, PP_ERR_INVALID, "FFV1 record: state transition %d", v);
            one[i] = (uint8_t)v;
        }
        for (int i = 1; i < 256; i++) {  // ff_ffv1_init_slice_state
            R.one_state[i] = one[i];
            R.zero_state[256 - i] = (uint8_t)(256 - one[i]);
        }
    }
    const int cs = r.symbol(st);
    R.bits = r.symbol(st);
    const int chroma = r.rac(st);
    R.hsub = r.symbol(st);
    R.vsub = r.symbol(st);
    const int alpha = r.rac(st);
    const int nh1 = r.symbol(st), nv1 = r.symbol(st);
    R.ntables = r.symbol(st);
    if (cs != 0 || !chroma || alpha)
        return fail(err, PP_ERR_UNSUPPORTED, "FFV1 record: colorspace %d chroma %d alpha %d (supported: YCbCr, chroma, no alpha)",
                    cs, chroma, alpha);
    if (R.bits < 8 || R.bits > 10 || R.hsub < 0 || R.hsub > 1 || R.vsub < 0 || R.vsub > 1)
        return fail(err, PP_ERR_UNSUPPORTED, "FFV1 record: %d bits, chroma shifts %d/%d", R.bits, R.hsub, R.vsub);
    if (nh1 < 0 || nv1 < 0 || nh1 >= 256 || nv1 >= 256)
        return fail(err, PP_ERR_INVALID, "FFV1 record: slice grid %dx%d", nh1 + 1, nv1 + 1);
    R.nh = nh1 + 1;
    R.nv = nv1 + 1;
    if (R.nh * R.nv > 256 || R.nh > w || R.nv > h)
        return fail(err, PP_ERR_INVALID, "FFV1 record: slice grid %dx%d", R.nh, R.nv);
    if (R.ntables < 1 || R.ntables > kFfv1MaxTables)
        return fail(err, PP_ERR_INVALID, "FFV1 record: %d quantisation table sets", R.ntables);
    for (int s = 0; s < R.ntables; s++) {  // read_quant_tables
        int64_t cc = 1;
        for (int t = 0; t < 5; t++) {
            uint8_t qs[kFfv1CtxBytes];
            std::memset(qs, 128, sizeof(qs));
            int16_t *q = R.quant[s][t];
            int i = 0, v = 0;
            for (; i < 128; v++) {
                const int run = r.symbol(qs);  // run length - 1
                if (run < 0 || run >= 128 - i)
                    return fail(err, PP_ERR_INVALID, "FFV1 record: quantisation table %d.%d", s, t);
                for (int k = 0; k <= run; k++) q[i++] = (int16_t)(cc * v);
            }
            for (i = 1; i < 128; i++) q[256 - i] = (int16_t)-q[i];
            q[128] = (int16_t)-q[127];
            cc *= 2 * v - 1;
            if (cc > 32768) return fail(err, PP_ERR_INVALID, "FFV1 record: quantisation set %d: too many contexts", s);
        }
        R.ctx_count[s] = (int)((cc + 1) / 2);
        R.max_ctx = std::max(R.max_ctx, R.ctx_count[s]);
    }
    uint8_t st2[kFfv1CtxBytes][kFfv1CtxBytes];
    std::memset(st2, 128, sizeof(st2));
    for (int s = 0; s < R.ntables; s++) {
        if (!r.rac(st)) continue;
        R.init[s].resize((size_t)R.ctx_count[s] * kFfv1CtxBytes);
        uint8_t *p = R.init[s].data();
        for (int j = 0; j < R.ctx_count[s]; j++)
            for (int k = 0; k < kFfv1CtxBytes; k++) {
                const int pred = j ? p[(j - 1) * kFfv1CtxBytes + k] : 128;
                const int d = r.ssymbol(st2[k], true, &bad);
                if (bad) return fail(err, PP_ERR_INVALID, "FFV1 record: initial states of set %d", s);
                p[j * kFfv1CtxBytes + k] = (uint8_t)((pred + d) & 0xFF);
            }
    }
    R.ec = r.symbol(st);
    if (R.ec < 0 || R.ec > 1) return fail(err, PP_ERR_INVALID, "FFV1 record: ec %d", R.ec);
    R.intra = R.micro > 2 ? r.symbol(st) : 0;
    if (R.intra < 0) return fail(err, PP_ERR_INVALID, "FFV1 record: intra %d", R.intra);
    *rec = R;
    return PP_OK;
}

int ffv1_keyframe_bit(const uint8_t *slice0, int64_t n) {
    // the first decision of the frame coder at state 128 (decode_frame):
    // range 0xFF00 splits at 0x7F80; ff_init_range_decoder clamps low to 0xFF00
    const int low = n >= 2 ? ((int)slice0[0] << 8) | slice0[1] : 0;
    return std::min(low, 0xFF00) >= 0x7F80 ? 1 : 0;
}

int ffv1_slice_table(const uint8_t *packets, const int64_t *frame_sizes, int nframes, int per, int ec,
                     int64_t *soff, int64_t *slen, int64_t *total, std::string *err) {
    if (nframes < 0 || per < 1 || (nframes > 0 && (!packets || !frame_sizes || !soff || !slen)))
        return fail(err, PP_ERR_INVALID, "null argument");
    const int trailer = 3 + 5 * (ec != 0);
    int64_t base = 0;
    for (int f = 0; f < nframes; ++f) {  // slices from the end of the packet (ffv1dec.c decode_frame)
        if (frame_sizes[f] < 0 || frame_sizes[f] > ((int64_t)1 << 40))
            return fail(err, PP_ERR_INVALID, "frame %d: size %lld", f, (long long)frame_sizes[f]);
        int64_t end = base + frame_sizes[f];
        for (int i = per - 1; i >= 0; --i) {
            if (end - base < trailer) return fail(err, PP_ERR_INVALID, "frame %d: slice %d trailer missing", f, i);
            const uint8_t *t = packets + end - trailer;
            const int64_t v = ((int64_t)t[0] << 16 | (int64_t)t[1] << 8 | t[2]) + trailer;
            if (i == 0 ? v != end - base : v > end - base)
                return fail(err, PP_ERR_INVALID, "frame %d: slice pointer chain broken at slice %d", f, i);
            end -= v;
            soff[(int64_t)f * per + i] = end;
            slen[(int64_t)f * per + i] = v;
        }
        base += frame_sizes[f];
    }
    if (total) *total = base;
    return PP_OK;
}

}  // namespace pp
