// FFV1 version 3 decoder on gfx950 (the decode
// half): reads AVPVS frame packets back into planar frames in HBM for the
// CPVS stage (create_cpvs decodes the FFV1 AVPVS, lib/ffmpeg.py:1149-1201).
//
// Same shape as the encoder (ffv1.hip): ONE LANE PER SLICE CHAIN.  A chain is
// one slice position over one GOP -- a keyframe and the inter frames after it,
// whose context states carry over from frame to frame (RFC 9043 4.5; FFmpeg's
// `-level 3 -coder 1 -context 1` AVPVS of lib/ffmpeg.py:993, :1047 has a GOP
// of 12); an intra stream (pixpath's own) has one-frame chains, so the batch
// is frames x slices lanes.  The host walks each packet's slice footers
// backwards (24-bit sizes, RFC 9043 4.8) into a slice table and reads each
// frame's keyframe bit to cut the GOPs; a GOP that starts before the batch
// continues from the states the previous call left (`carry`).  A lane checks
// its slices' CRC-32 parity, then per frame reads the keyframe bit (first
// slice), the slice header (position and per-plane quantisation table set,
// as FFmpeg's decode_slice_header), on a keyframe loads the record's initial
// states, decodes Y, Cb, Cr in raster order -- quantised context from the
// record's tables (LDS), median prediction, get_symbol through the slice's
// context states -- writing each sample straight into the destination planes,
// and finishes with the closing bit at state 129 and FFmpeg's end-of-slice
// position check.  Per-slice status: 0 ok, 1 CRC, 2 header, 3 end mismatch.
#include <algorithm>
#include <cstring>
#include <memory>
#include <vector>

#include "common.hpp"
#include "device.hpp"
#include "ffv1host.hpp"

namespace pp {

namespace {

constexpr size_t kLineLds = 160 * 1024 - 4096;  // LDS left for line buffers (gfx950: 160 KB per CU)

}  // namespace

struct Ffv1DecArgs {
    const uint8_t *pkt;
    const int64_t *soff, *slen;  // [nframes * per] slice start and length (trailer included)
    uint8_t *dst[3];
    int64_t ls[3], fs[3];
    int w, h, bytes, bits, hsub, vsub, nh, nv, per, nchains, ec;
    const int *gop;              // [nchains / per][3]: first frame, frames, 1 = starts at a keyframe (else carried states)
    int max_ctx;                 // state slots per plane set (the record's largest table set)
    int ntables;                 // quantisation table sets in LDS
    int ctx_count[kFfv1MaxTables];
    int init_off[kFfv1MaxTables];  // context offset of a set's initial states in `init`, -1: all 128
    int lpw;                     // chains (active lanes) per 64-lane workgroup
    int row_cap;                 // samples per lane and row in the LDS line buffers (>= widest slice row)
    int debug;                   // PIXPATH_FFV1_DEBUG (timing ablation only; the output is wrong):
                                 // 2 no CRC check
    int64_t state_bytes;         // per chain and half: 2 * max_ctx * 16
    uint8_t *states;             // hot halves [nchains / 64][2 * max_ctx][64][16]
    uint8_t *cold;               // cold halves, same layout
    int *status;                 // [nframes * per], zeroed by the host
    const uint8_t *tables;       // zero[256], one[256] (the record's), crc table, x^(8 * 2^j)
    const int16_t *quant;        // [ntables][5][256] (scaled)
    const uint4 *init;           // [contexts][hot 16 | cold 16] initial states, split as the state halves
    int qthr[5];                 // PIX: the first quantiser's thresholds (Ffv1Quant), unused ones 1024
};

// The slice's range decoder (rangecoder.h get_rac / refill) on register-held
// state: a symbol's state bytes come from the current context's 32-byte block
// in 8 VGPRs (all read before its first decision, updated bytes written after
// the last, so the LDS state-table lookups never sit on the low/range chain).
// The bytestream is read a dword at a time: `cur` holds the word at `pos`,
// and each sample issues the load of the following word into `nxt` before its
// state-block load (dec_prefetch), so a refill that enters that word takes it
// from a register whose load has completed with the block's.  A refill that
// enters any other word loads it there (the header, or a sample past two
// words).
struct Dec {
    uint32_t low, range;
    int pos, end;  // byte positions relative to the dword-aligned base `w`
    uint32_t cur, nxt;
    int nk;        // word index held in `nxt`
    const uint32_t *w;
};

__device__ __forceinline__ void dec_prefetch(Dec &d) {
    d.nk = (d.pos >> 2) + 1;
    d.nxt = d.w[d.nk];
}

__device__ __forceinline__ void dec_refill(Dec &d) {
    if (d.range < 0x100u) {
        d.range <<= 8;
        d.low <<= 8;
        if (d.pos < d.end) {
            d.low += (d.cur >> ((d.pos & 3) * 8)) & 0xFFu;
            d.pos++;
            if ((d.pos & 3) == 0) {
                if ((d.pos >> 2) == d.nk) d.cur = d.nxt;
                else d.cur = d.w[d.pos >> 2];
            }
        }
    }
}

// one decision with state value s; ns receives the next state value
__device__ __forceinline__ uint32_t dec_rac(Dec &d, uint32_t s, const uint8_t *tab, uint32_t &ns) {
    const uint32_t r1 = __umul24(d.range, s) >> 8;
    const uint32_t r0 = d.range - r1;
    const uint32_t bit = d.low >= r0 ? 1u : 0u;
    d.low -= bit ? r0 : 0u;
    d.range = bit ? r1 : r0;
    ns = tab[s | (bit << 8)];
    dec_refill(d);
    return bit;
}

__device__ __forceinline__ uint32_t dsget(const uint32_t (&b)[8], int k) { return (b[k >> 2] >> ((k & 3) * 8)) & 0xFFu; }
__device__ __forceinline__ void dsput(uint32_t (&b)[8], int k, uint32_t v) {
    b[k >> 2] = (b[k >> 2] & ~(0xFFu << ((k & 3) * 8))) | (v << ((k & 3) * 8));
}
__device__ __forceinline__ uint32_t dsget_dyn(const uint32_t (&b)[8], int k) {  // k in 8..23
    const int w = k >> 2;
    const uint32_t x = w == 2 ? b[2] : w == 3 ? b[3] : w == 4 ? b[4] : b[5];
    return (x >> ((k & 3) * 8)) & 0xFFu;
}
__device__ __forceinline__ void dsput_dyn(uint32_t (&b)[8], int k, uint32_t v) {
    const int w = k >> 2;
    const uint32_t sh = (k & 3) * 8, m = ~(0xFFu << sh), nv = v << sh;
    b[2] = w == 2 ? (b[2] & m) | nv : b[2];
    b[3] = w == 3 ? (b[3] & m) | nv : b[3];
    b[4] = w == 4 ? (b[4] & m) | nv : b[4];
    b[5] = w == 5 ? (b[5] & m) | nv : b[5];
}

// get_symbol (ffv1dec.c) for samples of <= 10 bits: exponent e <= 9, so
// every state index is used at most once per symbol; e >= 10 (not a <= 10-bit
// stream) sets `bad`.
template <bool SIGNED>
__device__ __forceinline__ int dec_symbol(Dec &d, uint32_t (&b)[8], const uint8_t *tab, bool &bad) {
    uint32_t n0;
    const uint32_t z = dec_rac(d, dsget(b, 0), tab, n0);
    uint32_t nu[10], nm[9], nsg = 0;
    int e = 0, a = 1;
    uint32_t neg = 0;
    if (!z) {
        bool go = true;
#pragma unroll
        for (int i = 0; i < 10; ++i)
            if (go) {
                if (dec_rac(d, dsget(b, 1 + i), tab, nu[i])) e = i + 1;
                else go = false;
            }
        if (go) bad = true;
#pragma unroll
        for (int i = 8; i >= 0; --i)
            if (i < e) a = 2 * a + (int)dec_rac(d, dsget(b, 22 + i), tab, nm[i]);
        if constexpr (SIGNED) neg = dec_rac(d, dsget_dyn(b, 11 + min(e, 9)), tab, nsg);
    }
    dsput(b, 0, n0);
    if (!z) {
#pragma unroll
        for (int i = 0; i < 10; ++i)
            if (i <= e) dsput(b, 1 + i, nu[i]);
#pragma unroll
        for (int i = 0; i < 9; ++i)
            if (i < e) dsput(b, 22 + i, nm[i]);
        if constexpr (SIGNED) dsput_dyn(b, 11 + min(e, 9), nsg);
    }
    return z ? 0 : (neg ? -a : a);
}

// A context's 32 state bytes split in two 16-byte halves.  HOT (the block
// loaded on every context switch): [0] zero flag, [1..5] exponent
// bits 0..4, [6..10] sign for e = 0..4, [11..14] mantissa bits 0..3 -- every
// state a residual below 32 in magnitude touches.  COLD (its own array):
// [0..4] exponent bits 5..9, [5..9] sign for e = 5..9, [10..14] mantissa bits
// 4..8, loaded only once a symbol's exponent reaches 5.
__device__ __forceinline__ uint32_t bget(const uint32_t (&b)[4], int k) { return (b[k >> 2] >> ((k & 3) * 8)) & 0xFFu; }
__device__ __forceinline__ void bput(uint32_t (&b)[4], int k, uint32_t v) {
    b[k >> 2] = (b[k >> 2] & ~(0xFFu << ((k & 3) * 8))) | (v << ((k & 3) * 8));
}

// get_symbol (ffv1dec.c) for samples of <= 10 bits: exponent e <= 9, so every
// state index is used at most once per symbol; e >= 10 (not a <= 10-bit
// stream) sets `bad`.  Decisions read the block as loaded and write the next
// states into a copy, so no decision waits on the previous one's state-table
// lookup (neighbouring state bytes share a dword).
template <bool SIGNED>
__device__ __forceinline__ int dec_symbol_split(Dec &d, uint32_t (&h)[4], uint8_t *cold, const uint8_t *tab, bool &bad) {
    const uint32_t h0[4] = {h[0], h[1], h[2], h[3]};
    uint32_t ns;
    const uint32_t z = dec_rac(d, bget(h0, 0), tab, ns);
    bput(h, 0, ns);
    if (z) return 0;
    int e = 0, a = 1;
    bool go = true;
#pragma unroll
    for (int i = 0; i < 5; ++i)
        if (go) {
            const uint32_t bit = dec_rac(d, bget(h0, 1 + i), tab, ns);
            bput(h, 1 + i, ns);
            if (bit) e = i + 1;
            else go = false;
        }
    uint32_t neg;
    if (go) {  // e >= 5: the cold half
        const uint4 x = *reinterpret_cast<const uint4 *>(cold);
        const uint32_t c0[4] = {x.x, x.y, x.z, x.w};
        uint32_t c[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int i = 5; i < 10; ++i)
            if (go) {
                const uint32_t bit = dec_rac(d, bget(c0, i - 5), tab, ns);
                bput(c, i - 5, ns);
                if (bit) e = i + 1;
                else go = false;
            }
        if (go) bad = true;
#pragma unroll
        for (int i = 8; i >= 4; --i)
            if (i < e) {
                a = 2 * a + (int)dec_rac(d, bget(c0, 10 + i - 4), tab, ns);
                bput(c, 10 + i - 4, ns);
            }
#pragma unroll
        for (int i = 3; i >= 0; --i) {
            a = 2 * a + (int)dec_rac(d, bget(h0, 11 + i), tab, ns);
            bput(h, 11 + i, ns);
        }
        neg = 0;
        if constexpr (SIGNED) {
            const int k = min(e, 9);  // sign state 5 + (k - 5) of the cold half
            const uint32_t sv = k == 5 ? bget(c0, 5) : k == 6 ? bget(c0, 6) : k == 7 ? bget(c0, 7) : k == 8 ? bget(c0, 8) : bget(c0, 9);
            neg = dec_rac(d, sv, tab, ns);
            if (k == 5) bput(c, 5, ns);
            else if (k == 6) bput(c, 6, ns);
            else if (k == 7) bput(c, 7, ns);
            else if (k == 8) bput(c, 8, ns);
            else bput(c, 9, ns);
        }
        *reinterpret_cast<uint4 *>(cold) = make_uint4(c[0], c[1], c[2], c[3]);
    } else {
#pragma unroll
        for (int i = 3; i >= 0; --i)
            if (i < e) {
                a = 2 * a + (int)dec_rac(d, bget(h0, 11 + i), tab, ns);
                bput(h, 11 + i, ns);
            }
        neg = 0;
        if constexpr (SIGNED) {  // sign state 6 + e, e in 0..4
            const uint32_t sv = e == 0 ? bget(h0, 6) : e == 1 ? bget(h0, 7) : e == 2 ? bget(h0, 8) : e == 3 ? bget(h0, 9) : bget(h0, 10);
            neg = dec_rac(d, sv, tab, ns);
            if (e == 0) bput(h, 6, ns);
            else if (e == 1) bput(h, 7, ns);
            else if (e == 2) bput(h, 8, ns);
            else if (e == 3) bput(h, 9, ns);
            else bput(h, 10, ns);
        }
    }
    return neg ? -a : a;
}

// a(x) b(x) mod P for the slice CRC's polynomial (CRC-32 IEEE, MSB first)
__device__ __forceinline__ uint32_t gf2_mulmod(uint32_t a, uint32_t b) {
    uint32_t r = 0;
#pragma unroll
    for (int i = 31; i >= 0; --i) {
        r = (r << 1) ^ ((r & 0x80000000u) ? 0x04C11DB7u : 0u);
        r ^= ((a >> i) & 1u) ? b : 0u;
    }
    return r;
}

__device__ __forceinline__ void dblk_load(uint32_t (&b)[8], const uint8_t *p) {
    const uint4 x = reinterpret_cast<const uint4 *>(p)[0], y = reinterpret_cast<const uint4 *>(p)[1];
    b[0] = x.x; b[1] = x.y; b[2] = x.z; b[3] = x.w; b[4] = y.x; b[5] = y.y; b[6] = y.z; b[7] = y.w;
}
__device__ __forceinline__ void dblk_store(uint8_t *p, const uint32_t (&b)[8]) {
    reinterpret_cast<uint4 *>(p)[0] = make_uint4(b[0], b[1], b[2], b[3]);
    reinterpret_cast<uint4 *>(p)[1] = make_uint4(b[4], b[5], b[6], b[7]);
}


__device__ __forceinline__ int dmedian3(int a, int b, int c) { return max(min(a, b), min(max(a, b), c)); }

// A pixpath-form first quantiser (ffv1host.cpp ffv1_quant: the number of
// thresholds <= |d|, odd-mirrored, scale 1) as ALU code: the only lookup that
// depends on the sample just decoded leaves LDS
__device__ __forceinline__ int dquant0(int d, const int (&thr)[5]) {  // d already & 0xFF
    const int m = d < 128 ? d : (d == 128 ? 127 : 256 - d);
    const int q = (m >= thr[0]) + (m >= thr[1]) + (m >= thr[2]) + (m >= thr[3]) + (m >= thr[4]);
    return d < 128 ? q : -q;
}

// Copy chain states (both halves, every context) between two slot arrays of
// the [slot / 64][nctx][64][16] layout: the GOP carried into the next decode.
__global__ __launch_bounds__(256) void ffv1_state_copy_kernel(const uint8_t *src, int64_t src_half, int src_slot0,
                                                              uint8_t *dst, int64_t dst_half, int dst_slot0, int nslots,
                                                              int nctx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per_half = (int64_t)nslots * nctx;
    if (i >= 2 * per_half) return;
    const int half = (int)(i / per_half);
    const int64_t r = i - half * per_half;
    const int slot = (int)(r % nslots), k = (int)(r / nslots);
    auto at = [&](int sl) { return (int64_t)(sl >> 6) * (64 * (int64_t)nctx * 16) + (int64_t)k * 1024 + (sl & 63) * 16; };
    const uint4 v = *reinterpret_cast<const uint4 *>(src + half * src_half + at(src_slot0 + slot));
    *reinterpret_cast<uint4 *>(dst + half * dst_half + at(dst_slot0 + slot)) = v;
}

// PIX: the record is pixpath's own 3-input set (first quantiser as ALU code,
// one LDS line row per lane); else the general 5-input context
// (ffv1_template.c get_context) over two line rows -- the row above and the
// row two above, which the current row overwrites in place (decode_plane's
// sample buffers).  A set whose inputs 4 and 5 are unused has all-zero tables
// there (read_quant_table: non-decreasing levels from 0), so the sum is the
// 3-input context.
template <int BYTES, bool PIX>
__global__ __launch_bounds__(64) void ffv1_decode_kernel(const Ffv1DecArgs a) {
    __shared__ uint8_t s_tab[512];  // zero[256], one[256]
    __shared__ uint32_t s_crc[256];
    __shared__ uint32_t s_xp[32];   // x^(8 * 2^j) mod P
    extern __shared__ __align__(16) int16_t s_dyn[];  // [ntables][5][256] quantisers, then [lpw][rows][row_cap] lines
    const int lane = threadIdx.x;
    for (int i = lane; i < 256; i += blockDim.x) {
        s_tab[i] = a.tables[i];
        s_tab[256 + i] = a.tables[256 + i];
        s_crc[i] = reinterpret_cast<const uint32_t *>(a.tables + 512)[i];
    }
    const int nq = a.ntables * 5 * 256;
    for (int i = lane; i < nq; i += blockDim.x) s_dyn[i] = a.quant[i];
    if (lane < 32) s_xp[lane] = reinterpret_cast<const uint32_t *>(a.tables + 1536)[lane];
    __syncthreads();
    const int c = blockIdx.x * a.lpw + lane;  // this lane's chain
    if (a.ec && !(PP_ABLATE(a.debug) & 2)) {
        // CRC-32 parity of each slice, trailer included, must leave 0.  The
        // whole wave checks one slice at a time: lane t takes the t-th 64th
        // of its bytes, and its remainder moves past the bytes after them
        // (times x^(8 m) mod P) before the XOR over the wave -- the CRC is
        // linear in the message.
        int bad_j = -1;
        for (int t = 0; t < a.lpw; ++t) {
            const int ct = blockIdx.x * a.lpw + t;
            if (ct >= a.nchains) break;
            const int kt = ct / a.per, st_ = ct - kt * a.per;
            const int f0t = a.gop[3 * kt], nft = a.gop[3 * kt + 1];
            for (int j = 0; j < nft; ++j) {
                const int64_t gj = (int64_t)(f0t + j) * a.per + st_;
                const uint8_t *const sj = a.pkt + a.soff[gj];
                const int nj = (int)a.slen[gj];
                const int C = (nj + 63) / 64;
                const int b0 = min(nj, lane * C), b1 = min(nj, b0 + C);
                uint32_t crc = 0;
#pragma unroll 8
                for (int i = b0; i < b1; ++i) crc = (crc << 8) ^ s_crc[(crc >> 24) ^ sj[i]];
                for (int k = 0, m = nj - b1; m; ++k, m >>= 1)
                    if (m & 1) crc = gf2_mulmod(crc, s_xp[k]);
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) crc ^= (uint32_t)__shfl_xor((int)crc, o, 64);
                if (lane == t && crc != 0 && bad_j < 0) bad_j = j;
            }
        }
        if (lane < a.lpw && c < a.nchains && bad_j >= 0) {
            const int kc = c / a.per;
            a.status[(int64_t)(a.gop[3 * kc] + bad_j) * a.per + (c - kc * a.per)] = 1;
            return;
        }
    }
    if (lane >= a.lpw || c >= a.nchains) return;
    const int kg = c / a.per, s = c - kg * a.per;
    const int f0 = a.gop[3 * kg], nf = a.gop[3 * kg + 1], key_start = a.gop[3 * kg + 2] & 1;
    uint16_t *const lines = reinterpret_cast<uint16_t *>(s_dyn + nq) + lane * a.row_cap * (PIX ? 1 : 2);
    // context states of 64 neighbouring chains interleaved by chain (as the
    // encoder's): context k of chain c at [c / 64][k][c % 64], so a context
    // that is hot in neighbouring slices -- the same picture content -- shares
    // their 128-B lines in L2 instead of one line per slice
    uint8_t *const st0 = a.states + (int64_t)(c >> 6) * (64 * a.state_bytes) + (c & 63) * 16;
    uint8_t *const co0 = a.cold + (int64_t)(c >> 6) * (64 * a.state_bytes) + (c & 63) * 16;
    constexpr int kCtxStride = 64 * 16;
    const int mask = (1 << a.bits) - 1;
    for (int j = 0; j < nf; ++j) {
        const int64_t g = (int64_t)(f0 + j) * a.per + s;  // (frame, slice) of this step
        const uint8_t *const sb = a.pkt + a.soff[g];
        const int64_t n = a.slen[g];
        Dec d;
        {
            // pkt is 256-B aligned: the slice's misalignment is its offset's
            const int off = (int)(a.soff[g] & 3);
            d.w = reinterpret_cast<const uint32_t *>(sb - off);
            d.end = off + (int)n;
            d.range = 0xFF00;
            d.low = n >= 2 ? ((uint32_t)sb[0] << 8) | sb[1] : 0;
            d.pos = off + 2;
            if (d.low >= 0xFF00u) { d.low = 0xFF00u; d.end = d.pos; }
            d.cur = d.w[d.pos >> 2];
            dec_prefetch(d);
        }
        uint32_t dummy;
        const bool key = j == 0 && key_start;
        if (s == 0 && dec_rac(d, 128, s_tab, dummy) != (key ? 1u : 0u)) {  // keyframe bit
            a.status[g] = 2;
            return;
        }
        bool bad = false;
        int hv[9];
        {
            uint32_t hb[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) hb[i] = 0x80808080u;
#pragma unroll
            for (int i = 0; i < 9; ++i) hv[i] = dec_symbol<false>(d, hb, s_tab, bad);
        }
        const int sx = hv[0], sy = hv[1], sw = hv[2] + 1, sh = hv[3] + 1;
        if (bad || sx < 0 || sy < 0 || sx > a.nh - sw || sy > a.nv - sh || hv[4] < 0 || hv[4] >= a.ntables ||
            hv[5] < 0 || hv[5] >= a.ntables || (PIX && (hv[4] || hv[5]))) {
            a.status[g] = 2;
            return;
        }
        const int x0 = (int)((int64_t)sx * a.w / a.nh), x1 = (int)((int64_t)(sx + sw) * a.w / a.nh);
        const int y0 = (int)((int64_t)sy * a.h / a.nv), y1 = (int)((int64_t)(sy + sh) * a.h / a.nv);
        if (x1 - x0 > a.row_cap) {  // wider than this grid's slices
            a.status[g] = 2;
            return;
        }
        if (key) {  // ff_ffv1_clear_slice_state: the set's initial states (the host primed 128s)
            for (int p = 0; p < 2; ++p) {
                const int ti = hv[4 + p], io = a.init_off[ti];
                if (io < 0) continue;
                for (int q = 0; q < a.ctx_count[ti]; ++q) {
                    const uint4 hot = a.init[2 * (int64_t)(io + q)], cold = a.init[2 * (int64_t)(io + q) + 1];
                    *reinterpret_cast<uint4 *>(st0 + (p * a.max_ctx + q) * kCtxStride) = hot;
                    *reinterpret_cast<uint4 *>(co0 + (p * a.max_ctx + q) * kCtxStride) = cold;
                }
            }
        }
        // the block of context 0 in registers (every switch writes the held
        // block back, so it must start as the stored one)
        int cur_key = 0;
        uint32_t blk[4];
        {
            const uint4 b0 = *reinterpret_cast<const uint4 *>(st0);
            blk[0] = b0.x; blk[1] = b0.y; blk[2] = b0.z; blk[3] = b0.w;
        }
        for (int p = 0; p < 3; p++) {
            const int pw = p ? ((x1 - x0) + (1 << a.hsub) - 1) >> a.hsub : x1 - x0;
            const int ph = p ? ((y1 - y0) + (1 << a.vsub) - 1) >> a.vsub : y1 - y0;
            const int px0 = p ? x0 >> a.hsub : x0, py0 = p ? y0 >> a.vsub : y0;
            uint8_t *dp = p == 0 ? a.dst[0] : p == 1 ? a.dst[1] : a.dst[2];
            const int64_t ls = p == 0 ? a.ls[0] : p == 1 ? a.ls[1] : a.ls[2];
            const int64_t fs = p == 0 ? a.fs[0] : p == 1 ? a.fs[1] : a.fs[2];
            uint8_t *base = dp + (int64_t)(f0 + j) * fs + (int64_t)py0 * ls + (int64_t)px0 * BYTES;
            const int key0 = p ? a.max_ctx : 0;
            const int16_t *const q = s_dyn + hv[4 + (p ? 1 : 0)] * (5 * 256);
            auto put = [&](uint8_t *r, int xx, int vv) {
                if (BYTES == 2)
                    reinterpret_cast<uint16_t *>(r)[xx] = (uint16_t)vv;
                else
                    r[xx] = (uint8_t)vv;
            };
            int pv = 0;
            int T0prev = 0;  // PIX: the row above's first sample, one row later: TL at a row start
            // general: `up` holds the row above, `two` the row two above, which
            // the current row overwrites sample by sample (TT read first)
            uint16_t *up = lines, *two = PIX ? lines : lines + a.row_cap;
            for (int y = 0; y < ph; y++) {
                uint8_t *row = base + (int64_t)y * ls;
                // the row above is never read for the first row (nor the row two above for the first two)
                int T = y > 0 ? up[0] : 0;
                int TL;
                if constexpr (PIX) {
                    TL = y > 1 ? T0prev : 0;
                    T0prev = T;
                } else {
                    TL = y > 1 ? two[0] : 0;
                }
                int L = T, LL = 0;
                // the row above two columns ahead, read a sample early
                int TR = pw > 1 ? (y > 0 ? up[1] : 0) : T;
                int TT = (!PIX && y > 1) ? two[0] : 0;
                for (int x = 0; x < pw; x++) {
                    const int nTR = x + 2 < pw ? (y > 0 ? up[x + 2] : 0) : TR;
                    int nTT = 0;
                    if constexpr (!PIX) nTT = (y > 1 && x + 1 < pw) ? two[x + 1] : 0;
                    int ctx;
                    if constexpr (PIX)
                        ctx = dquant0((L - TL) & 0xFF, a.qthr) + q[256 + ((TL - T) & 0xFF)] + q[512 + ((T - TR) & 0xFF)];
                    else
                        ctx = q[(L - TL) & 0xFF] + q[256 + ((TL - T) & 0xFF)] + q[512 + ((T - TR) & 0xFF)] +
                              q[768 + ((LL - L) & 0xFF)] + q[1024 + ((TT - T) & 0xFF)];
                    const bool neg = ctx < 0;
                    if (neg) ctx = -ctx;
                    const int key = key0 + ctx;
                    dec_prefetch(d);
                    // Branch-free: memory operations complete in issue order, so the
                    // block load goes out before the previous sample's store and the
                    // write-back of the current block, and waiting for it does not
                    // wait for their acks.  Same context: the load is stale and the
                    // registers are kept.
                    {
                        const uint4 nb = *reinterpret_cast<const uint4 *>(st0 + key * kCtxStride);
                        // (x = 0: the previous row's last sample lands on row[0] until x = 1 rewrites it)
                        put(row, max(x - 1, 0), pv);
                        *reinterpret_cast<uint4 *>(st0 + cur_key * kCtxStride) = make_uint4(blk[0], blk[1], blk[2], blk[3]);
                        const bool same = key == cur_key;
                        blk[0] = same ? blk[0] : nb.x;
                        blk[1] = same ? blk[1] : nb.y;
                        blk[2] = same ? blk[2] : nb.z;
                        blk[3] = same ? blk[3] : nb.w;
                        cur_key = key;
                    }
                    int diff = dec_symbol_split<true>(d, blk, co0 + cur_key * kCtxStride, s_tab, bad);
                    if (neg) diff = -diff;
                    const int v = (dmedian3(L, L + T - TL, T) + diff) & mask;
                    pv = v;  // stored during the next sample, after its block load
                    two[x] = (uint16_t)v;  // PIX: `two` is the one line (x is no longer T or TR)
                    TL = T;
                    T = TR;
                    TR = nTR;
                    LL = L;
                    L = v;
                    TT = nTT;
                }
                if (pw > 0) put(row, pw - 1, pv);
                if constexpr (!PIX) {
                    uint16_t *t = up;
                    up = two;
                    two = t;
                }
            }
        }
        *reinterpret_cast<uint4 *>(st0 + cur_key * kCtxStride) = make_uint4(blk[0], blk[1], blk[2], blk[3]);
        (void)dec_rac(d, 129, s_tab, dummy);  // the closing bit at state 129
        const int st = bad ? 2 : ((d.end - d.pos) - 2 - 5 * (a.ec != 0)) != 0 ? 3 : 0;
        if (st) {
            a.status[g] = st;
            return;
        }
    }
}

}  // namespace pp

using namespace pp;

struct pp_ffv1_dec {
    pp_ctx *ctx = nullptr;
    int w = 0, h = 0, max_frames = 0;
    Ffv1Record rec;
    bool pix = false;  // pixpath's own 3-input set (ALU first quantiser, one line row)
    Ffv1Quant pq;      // its thresholds
    uint8_t *pkt = nullptr, *states = nullptr, *tables = nullptr, *carry = nullptr;
    int64_t pkt_cap = 0, *soff = nullptr, *slen = nullptr;
    int *gop = nullptr;
    int row_cap = 0;  // widest slice row, rounded to 8 samples
    int lpw = 16;     // chains per workgroup: 16, fewer when their line buffers would not fit the LDS
    size_t lds = 0;   // dynamic LDS per workgroup at lpw: quantisers + line rows
    int *status = nullptr;
    int16_t *dquant = nullptr;
    uint4 *dinit = nullptr;
    int init_off[kFfv1MaxTables];
    // decode workspace, grown on demand to what a call needs (a
    // record with thousands of contexts no longer reserves per * max_frames
    // chain slots up front -- a GOP-12 stream needs a twelfth of them)
    int64_t slots = 0;        // chain state slots allocated (64-aligned)
    int64_t ns_cap = 0;       // slice entries (soff / slen / status)
    int64_t gop_cap = 0;      // GOP entries
    bool carry_valid = false; // `carry` holds the last GOP's states of the previous decode
    std::vector<uint8_t> extra;  // the configuration record (a group decode needs equal ones)
};

namespace {

// a context's 32 FFmpeg state bytes -> the HOT | COLD halves of the decoder
// (dec_symbol_split): HOT [0] zero, [1..5] exponent 0..4, [6..10] sign e = 0..4,
// [11..14] mantissa 0..3; COLD [0..4] exponent 5..9, [5..9] sign e = 5..9,
// [10..14] mantissa 4..8 (states 21 and 31 serve > 10-bit samples only)
void split_states(const uint8_t *st, uint8_t hot[16], uint8_t cold[16]) {
    std::memset(hot, 128, 16);
    std::memset(cold, 128, 16);
    hot[0] = st[0];
    for (int i = 0; i < 5; ++i) {
        hot[1 + i] = st[1 + i];
        hot[6 + i] = st[11 + i];
        cold[i] = st[6 + i];
        cold[5 + i] = st[16 + i];
        cold[10 + i] = st[26 + i];
    }
    for (int i = 0; i < 4; ++i) hot[11 + i] = st[22 + i];
}

// A record of pixpath's form: one set of 3 inputs whose quantisers are one
// threshold quantiser (Ffv1Quant, up to 5 thresholds) at scales 1, L, L^2 --
// what pixpath's encoder writes, whichever thresholds it chose.  *q gets the
// thresholds (the kernel's ALU first quantiser).
bool pixpath_tables(const Ffv1Record &r, Ffv1Quant *q) {
    if (r.ntables != 1) return false;
    Ffv1Quant t;
    t.n = 0;
    for (int i = 1; i < 128; ++i) {
        const int d = r.quant[0][0][i] - r.quant[0][0][i - 1];
        if (d < 0 || d > 1 || (d == 1 && t.n == 5)) return false;
        if (d == 1) t.thr[t.n++] = i;
    }
    if (r.quant[0][0][0] != 0) return false;
    const int L = t.levels();
    for (int i = 0; i < 256; ++i)
        if (r.quant[0][0][i] != ffv1_quant(i, t) || r.quant[0][1][i] != L * ffv1_quant(i, t) ||
            r.quant[0][2][i] != L * L * ffv1_quant(i, t) || r.quant[0][3][i] || r.quant[0][4][i])
            return false;
    *q = t;
    return true;
}

}  // namespace

extern "C" int pp_ffv1_decoder_create(pp_ctx *ctx, const uint8_t *extra, int extra_size, int w, int h,
                                      int max_frames, pp_ffv1_dec **out) {
    if (!out || !extra) PP_FAIL(PP_ERR_INVALID, "null argument");
    *out = nullptr;
    if (w < 2 || h < 2 || max_frames < 1) PP_FAIL(PP_ERR_INVALID, "bad size %dx%d / max_frames %d", w, h, max_frames);
    std::unique_ptr<pp_ffv1_dec> D(new pp_ffv1_dec());
    std::string err;
    if (int rc = ffv1_parse_record(extra, extra_size, w, h, &D->rec, &err)) PP_FAIL(rc, "%s", err.c_str());
    const Ffv1Record &R = D->rec;
    if (R.bits != 8 && R.bits != 10) PP_FAIL(PP_ERR_UNSUPPORTED, "FFV1 decoder: %d-bit samples (8 or 10)", R.bits);
    if (R.hsub == 0 && R.vsub == 1) PP_FAIL(PP_ERR_UNSUPPORTED, "FFV1 decoder: 4:4:0 chroma");
    D->ctx = ctx; D->w = w; D->h = h; D->max_frames = max_frames;
    D->pix = pixpath_tables(R, &D->pq);
    int wmax = 0;
    for (int i = 0; i < R.nh; ++i)
        wmax = std::max(wmax, (int)((int64_t)(i + 1) * w / R.nh - (int64_t)i * w / R.nh));
    D->row_cap = (wmax + 7) / 8 * 8;
    const size_t qbytes = (size_t)R.ntables * 5 * 256 * 2, rows = D->pix ? 1 : 2;
    const size_t per_lane = (size_t)D->row_cap * 2 * rows;
    D->lpw = qbytes + per_lane > kLineLds
                 ? 0
                 : (int)std::min<size_t>((size_t)ffv1_lanes_per_wave(16), (kLineLds - qbytes) / per_lane);
    if (D->lpw < 1)
        PP_FAIL(PP_ERR_UNSUPPORTED, "FFV1 decoder: %d-sample slice rows exceed the LDS line buffer", wmax);
    int ninit = 0;
    for (int t = 0; t < R.ntables; ++t) {
        D->init_off[t] = R.init[t].empty() ? -1 : ninit;
        ninit += R.init[t].empty() ? 0 : R.ctx_count[t];
    }
    if (!ctx) {
        *out = D.release();
        return PP_OK;
    }
    const int per = R.nh * R.nv;
    D->extra.assign(extra, extra + extra_size);
    const int64_t chalf = 2 * (int64_t)R.max_ctx * 16 * ((per + 63) / 64 * 64);
    PP_HIP(hipSetDevice(ctx->device));
    PP_HIP(hipMalloc(&D->carry, 2 * chalf));  // the decode workspace itself is allocated by the first decode
    PP_HIP(hipMalloc(&D->tables, 512 + 1024 + 128));
    PP_HIP(hipMalloc(&D->dquant, qbytes));
    uint8_t tab[512 + 1024 + 128];
    std::memcpy(tab, R.zero_state, 256);
    std::memcpy(tab + 256, R.one_state, 256);
    crc_table(reinterpret_cast<uint32_t *>(tab + 512));
    {  // x^(8 * 2^j) mod P by squaring, from x^8
        uint32_t *xp = reinterpret_cast<uint32_t *>(tab + 1536);
        auto mulmod = [](uint32_t x, uint32_t y) {
            uint32_t r = 0;
            for (int i = 31; i >= 0; --i) {
                r = (r << 1) ^ ((r & 0x80000000u) ? 0x04C11DB7u : 0u);
                if ((x >> i) & 1u) r ^= y;
            }
            return r;
        };
        xp[0] = 0x100u;
        for (int j = 1; j < 32; ++j) xp[j] = mulmod(xp[j - 1], xp[j - 1]);
    }
    PP_HIP(hipMemcpy(D->tables, tab, sizeof(tab), hipMemcpyHostToDevice));
    PP_HIP(hipMemcpy(D->dquant, R.quant, qbytes, hipMemcpyHostToDevice));
    if (ninit) {
        std::vector<uint8_t> split((size_t)ninit * 32);
        for (int t = 0; t < R.ntables; ++t)
            for (int k = 0; D->init_off[t] >= 0 && k < R.ctx_count[t]; ++k) {
                uint8_t *o = split.data() + (size_t)(D->init_off[t] + k) * 32;
                split_states(R.init[t].data() + (size_t)k * 32, o, o + 16);
            }
        PP_HIP(hipMalloc(&D->dinit, split.size()));
        PP_HIP(hipMemcpy(D->dinit, split.data(), split.size(), hipMemcpyHostToDevice));
    }
    *out = D.release();
    return PP_OK;
}

extern "C" int pp_ffv1_decoder_destroy(pp_ffv1_dec *D) {
    if (!D) return PP_OK;
    for (void *p : {(void *)D->pkt, (void *)D->states, (void *)D->carry, (void *)D->soff, (void *)D->slen,
                    (void *)D->status, (void *)D->gop, (void *)D->tables, (void *)D->dquant, (void *)D->dinit})
        if (p) (void)hipFree(p);
    delete D;
    return PP_OK;
}

extern "C" int pp_ffv1_decoder_geometry(const pp_ffv1_dec *D, int *slices_per_workgroup, int *row_cap) {
    if (!D || !slices_per_workgroup || !row_cap) PP_FAIL(PP_ERR_INVALID, "null argument");
    *slices_per_workgroup = D->lpw;
    *row_cap = D->row_cap;
    return PP_OK;
}

extern "C" int pp_ffv1_decoder_slices(const pp_ffv1_dec *D, int *slices_h, int *slices_v) {
    if (!D || !slices_h || !slices_v) PP_FAIL(PP_ERR_INVALID, "null argument");
    *slices_h = D->rec.nh;
    *slices_v = D->rec.nv;
    return PP_OK;
}

// Format of the decoded frames (PP_FMT_*), from the configuration record.
extern "C" int pp_ffv1_decoder_format(const pp_ffv1_dec *D) {
    if (!D) PP_FAIL(PP_ERR_INVALID, "null decoder");
    const Ffv1Record &R = D->rec;
    if (R.hsub == 0) return R.bits == 8 ? PP_FMT_YUV444P : PP_FMT_YUV444P10LE;
    if (R.bits == 8) return R.vsub ? PP_FMT_YUV420P : PP_FMT_YUV422P;
    return R.vsub ? PP_FMT_YUV420P10LE : PP_FMT_YUV422P10LE;
}

extern "C" int pp_ffv1_decoder_info(const pp_ffv1_dec *D, int *info, int n) {
    if (!D || !info || n < 0) PP_FAIL(PP_ERR_INVALID, "null argument");
    const Ffv1Record &R = D->rec;
    int has_init = 0;
    for (int t = 0; t < R.ntables; ++t) has_init |= (!R.init[t].empty()) << t;
    const int v[] = {R.micro, R.coder, R.ntables, R.max_ctx, R.intra, R.ec, has_init, D->pix ? 1 : 0};
    const int k = std::min<int>(n, (int)(sizeof(v) / sizeof(v[0])));
    for (int i = 0; i < k; ++i) info[i] = v[i];
    return k;
}

extern "C" int pp_ffv1_decoder_reset(pp_ffv1_dec *D) {
    if (!D) PP_FAIL(PP_ERR_INVALID, "null decoder");
    D->carry_valid = false;
    return PP_OK;
}

namespace {

// grow a device array to at least `need` elements (the decode is synchronous,
// so no earlier launch still uses the old one)
template <typename T>
hipError_t grow(T **p, int64_t *cap, int64_t need) {
    if (need <= *cap) return hipSuccess;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipError_t e = hipMalloc(p, sizeof(T) * need)) return e;
    *cap = need;
    return hipSuccess;
}

}  // namespace

// One launch over the slice chains of n streams of one configuration record
// (decs[k] decodes stream k: its packets, sizes and frame count; its carried
// GOP states in and out).  Stream k's frames land at dst frames
// [sum nframes[<k], ...).  The chains of one stream are few when its GOPs are
// long (FFmpeg's GOP 12 at 2x2 slices: 200 per 600 frames, one lane each), so
// several streams side by side are what fill the SIMDs.  decs[0] owns the
// launch workspace.
static int decode_group(pp_ffv1_dec *const *decs, int n, const uint8_t *const *packets,
                        const int64_t *const *frame_sizes, const int *nframes, const pp_frames *dst, void *stream) {
    if (!decs || n < 1 || !packets || !frame_sizes || !nframes || !dst) PP_FAIL(PP_ERR_INVALID, "null argument");
    pp_ffv1_dec *D = decs[0];
    for (int k = 0; k < n; ++k) {
        const pp_ffv1_dec *E = decs[k];
        if (!E || !packets[k] || !frame_sizes[k] || nframes[k] < 0) PP_FAIL(PP_ERR_INVALID, "null argument (stream %d)", k);
        if (!E->ctx) PP_FAIL(PP_ERR_INVALID, "host-only decoder cannot decode");
        if (nframes[k] > E->max_frames) PP_FAIL(PP_ERR_INVALID, "%d frames > max_frames %d", nframes[k], E->max_frames);
        for (int j = 0; j < k; ++j)
            if (decs[j] == E) PP_FAIL(PP_ERR_INVALID, "decoder of stream %d given twice", k);
        if (E->ctx != D->ctx || E->w != D->w || E->h != D->h || E->extra != D->extra)
            PP_FAIL(PP_ERR_INVALID, "stream %d: a group decode needs one configuration record, size and context", k);
    }
    const Ffv1Record &R = D->rec;
    hipStream_t st = static_cast<hipStream_t>(stream);
    PP_HIP(hipSetDevice(D->ctx->device));
    const int per = R.nh * R.nv;
    int64_t ftot = 0;
    for (int k = 0; k < n; ++k) ftot += nframes[k];
    if (ftot == 0) return PP_OK;
    const int64_t ns = per * ftot;
    std::vector<int64_t> soff(ns), slen(ns), bytes(n);
    std::vector<int> gop, first_gop(n), ngop(n);
    std::vector<char> carry_in(n);
    std::string err;
    int64_t base = 0, f0 = 0;
    for (int k = 0; k < n; ++k) {  // slice tables and GOPs, stream by stream
        pp_ffv1_dec *E = decs[k];
        carry_in[k] = E->carry_valid;
        first_gop[k] = (int)gop.size() / 3;
        const int nf = nframes[k];
        if (nf == 0) continue;
        E->carry_valid = false;  // until this decode has succeeded
        int64_t sb = 0;
        if (int rc = ffv1_slice_table(packets[k], frame_sizes[k], nf, per, R.ec, soff.data() + f0 * per,
                                      slen.data() + f0 * per, &sb, &err))
            PP_FAIL(rc, "stream %d: %s", k, err.c_str());
        for (int64_t i = f0 * per; i < (f0 + nf) * per; ++i) soff[i] += base;
        for (int f = 0; f < nf; ++f) {  // a keyframe starts a GOP; frame 0 without one continues the carried one
            const int64_t s0 = (f0 + f) * per;
            const int key = ffv1_keyframe_bit(packets[k] + soff[s0] - base, slen[s0]);
            if (f == 0 || key) {
                if (f == 0 && !key && !carry_in[k])
                    PP_FAIL(PP_ERR_INVALID, "stream %d: frame 0 is not a keyframe and no earlier frame of its GOP "
                                            "was decoded", k);
                gop.insert(gop.end(), {(int)(f0 + f), 0, key});
            }
            gop[gop.size() - 2]++;
        }
        ngop[k] = (int)gop.size() / 3 - first_gop[k];
        bytes[k] = sb;
        base += (sb + 63) & ~int64_t(63);
        f0 += nf;
    }
    const int ngops = (int)gop.size() / 3, nchains = ngops * per;
    if (base > D->pkt_cap) {
        if (D->pkt) PP_HIP(hipFree(D->pkt));
        D->pkt = nullptr;
        D->pkt_cap = 0;
        PP_HIP(hipMalloc(&D->pkt, base + 64));  // the bytestream window reads up to 8 B past a slice
        D->pkt_cap = base;
    }
    const int64_t sb = 2 * (int64_t)R.max_ctx * 16;  // one half, per chain
    const int64_t need_slots = ((int64_t)nchains + 63) / 64 * 64;
    if (need_slots > D->slots) {
        if (D->states) PP_HIP(hipFree(D->states));
        D->states = nullptr;
        D->slots = 0;
        PP_HIP(hipMalloc(&D->states, 2 * sb * need_slots));  // both halves
        D->slots = need_slots;
    }
    if (ns > D->ns_cap) {  // soff / slen / status share one capacity
        int64_t c = 0;
        D->ns_cap = 0;
        PP_HIP(grow(&D->soff, &c, ns));
        c = 0;
        PP_HIP(grow(&D->slen, &c, ns));
        c = 0;
        PP_HIP(grow(&D->status, &c, ns));
        D->ns_cap = ns;
    }
    PP_HIP(grow(&D->gop, &D->gop_cap, (int64_t)gop.size()));
    for (int64_t k = 0, off = 0; k < n; off += (bytes[k] + 63) & ~int64_t(63), ++k)
        if (bytes[k]) PP_HIP(hipMemcpyAsync(D->pkt + off, packets[k], bytes[k], hipMemcpyHostToDevice, st));
    PP_HIP(hipMemcpyAsync(D->soff, soff.data(), sizeof(int64_t) * ns, hipMemcpyHostToDevice, st));
    PP_HIP(hipMemcpyAsync(D->slen, slen.data(), sizeof(int64_t) * ns, hipMemcpyHostToDevice, st));
    PP_HIP(hipMemcpyAsync(D->gop, gop.data(), sizeof(int) * gop.size(), hipMemcpyHostToDevice, st));
    PP_HIP(hipMemsetAsync(D->status, 0, sizeof(int) * ns, st));
    const int64_t half = sb * D->slots, used = sb * need_slots;
    const int64_t chalf = sb * ((per + 63) / 64 * 64);
    PP_HIP(hipMemsetAsync(D->states, 128, used, st));
    PP_HIP(hipMemsetAsync(D->states + half, 128, used, st));
    auto copy_states = [&](const uint8_t *src, int64_t sh, int s0, uint8_t *dstp, int64_t dh, int d0) {
        const int64_t m = 2 * (int64_t)per * 2 * R.max_ctx;
        hipLaunchKernelGGL(ffv1_state_copy_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, src, sh, s0,
                           dstp, dh, d0, per, 2 * R.max_ctx);
        return hipGetLastError();
    };
    for (int k = 0; k < n; ++k)  // a stream whose first GOP continues its carried states
        if (ngop[k] && !gop[3 * first_gop[k] + 2])
            PP_HIP(copy_states(decs[k]->carry, chalf, 0, D->states, half, first_gop[k] * per));
    Ffv1DecArgs a{};
    a.pkt = D->pkt; a.soff = D->soff; a.slen = D->slen;
    for (int p = 0; p < 3; ++p) {
        a.dst[p] = static_cast<uint8_t *>(dst->data[p]);
        a.ls[p] = dst->linesize[p];
        a.fs[p] = dst->frame_stride[p];
    }
    a.w = D->w; a.h = D->h; a.bytes = R.bits > 8 ? 2 : 1; a.bits = R.bits; a.hsub = R.hsub; a.vsub = R.vsub;
    a.nh = R.nh; a.nv = R.nv; a.per = per; a.nchains = nchains; a.ec = R.ec; a.gop = D->gop;
    a.max_ctx = R.max_ctx; a.ntables = R.ntables;
    for (int t = 0; t < kFfv1MaxTables; ++t) {
        a.ctx_count[t] = t < R.ntables ? R.ctx_count[t] : 0;
        a.init_off[t] = t < R.ntables ? D->init_off[t] : -1;
    }
    a.state_bytes = sb;
    a.states = D->states; a.cold = D->states + half; a.status = D->status; a.tables = D->tables; a.quant = D->dquant;
    for (int k = 0; k < 5; ++k) a.qthr[k] = k < D->pq.n ? D->pq.thr[k] : 1024;
    a.init = D->dinit;
    // chains per workgroup: the LDS bound, spread over the CUs when chains are few (long GOPs)
    a.lpw = std::max(1, std::min(D->lpw, (nchains + D->ctx->cus - 1) / std::max(1, D->ctx->cus)));
    if (const char *e = PP_KNOB("PIXPATH_FFV1_DEBUG")) a.debug = std::atoi(e);
    a.row_cap = D->row_cap;
    static const hipError_t attr = [] {
        const void *fns[4] = {reinterpret_cast<const void *>(ffv1_decode_kernel<1, false>),
                              reinterpret_cast<const void *>(ffv1_decode_kernel<1, true>),
                              reinterpret_cast<const void *>(ffv1_decode_kernel<2, false>),
                              reinterpret_cast<const void *>(ffv1_decode_kernel<2, true>)};
        for (const void *f : fns)
            if (hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLineLds))
                return e;
        return hipSuccess;
    }();
    PP_HIP(attr);
    const dim3 grid((nchains + a.lpw - 1) / a.lpw), block(64);
    const size_t lds = (size_t)R.ntables * 5 * 256 * 2 + (size_t)a.lpw * D->row_cap * 2 * (D->pix ? 1 : 2);
    if (a.bytes == 2 && D->pix)
        hipLaunchKernelGGL((ffv1_decode_kernel<2, true>), grid, block, lds, st, a);
    else if (a.bytes == 2)
        hipLaunchKernelGGL((ffv1_decode_kernel<2, false>), grid, block, lds, st, a);
    else if (D->pix)
        hipLaunchKernelGGL((ffv1_decode_kernel<1, true>), grid, block, lds, st, a);
    else
        hipLaunchKernelGGL((ffv1_decode_kernel<1, false>), grid, block, lds, st, a);
    PP_HIP(hipGetLastError());
    // each stream's last GOP states, for its next decode that continues it
    for (int k = 0; k < n; ++k)
        if (ngop[k]) PP_HIP(copy_states(D->states, half, (first_gop[k] + ngop[k] - 1) * per, decs[k]->carry, chalf, 0));
    std::vector<int> status(ns);
    PP_HIP(hipMemcpyAsync(status.data(), D->status, sizeof(int) * ns, hipMemcpyDeviceToHost, st));
    PP_HIP(hipStreamSynchronize(st));
    static const char *what[] = {"ok", "slice CRC mismatch", "bad slice header", "bytestream end mismatch"};
    for (int64_t i = 0, fk = 0, k = 0; i < ns; ++i) {
        while (k < n && i >= (fk + nframes[k]) * per) fk += nframes[k++];
        if (status[i])
            PP_FAIL(PP_ERR_INVALID, "%sframe %d slice %d: %s", n > 1 ? ("stream " + std::to_string(k) + ": ").c_str() : "",
                    (int)(i / per - fk), (int)(i % per), what[std::min(status[i], 3)]);
    }
    for (int k = 0; k < n; ++k)
        if (nframes[k]) decs[k]->carry_valid = true;
    return PP_OK;
}

extern "C" int pp_ffv1_decode(pp_ffv1_dec *D, const uint8_t *packets, const int64_t *frame_sizes, int nframes,
                              const pp_frames *dst, void *stream) {
    if (!D || !packets || !frame_sizes || !dst || nframes < 0) PP_FAIL(PP_ERR_INVALID, "null argument");
    return decode_group(&D, 1, &packets, &frame_sizes, &nframes, dst, stream);
}

extern "C" int pp_ffv1_decode_group(pp_ffv1_dec *const *decs, int n, const uint8_t *const *packets,
                                    const int64_t *const *frame_sizes, const int *nframes, const pp_frames *dst,
                                    void *stream) {
    return decode_group(decs, n, packets, frame_sizes, nframes, dst, stream);
}
