// FFV1 version 3 intra encoder on gfx950: the
// AVPVS intermediate the reference writes with
// `-c:v ffv1 -threads 4 -level 3 -coder 1 -context 1 -slicecrc 1`
// (lib/ffmpeg.py:993, :1047).  Bitstream per RFC 9043 / FFmpeg 7.0 ffv1enc.c;
// the encoder's choices (range coder with the default state table, a 3-input
// threshold quantisation set per bit depth -- ffv1_default_quant: 63 contexts
// at 10 bits, 172 at 8 -- every frame a keyframe, caller-chosen slice grid,
// slice CRCs) are listed in oracle/ffv1_oracle.c and DESIGN.md.
//
// GPU shape: the range coder of a slice is one serial dependency chain (each
// binary decision updates `low/range` and an adaptive state byte), so the
// unit of parallelism is the slice: ONE LANE PER SLICE, every slice of every
// frame of the batch at once (600 frames x 64 slices = 38,400 lanes).  Only
// the coder itself is serial, so the encode is split in four launches:
//   ffv1_model_kernel   data-parallel, one thread per token: the context
//                       (quantised L-TL, TL-T, T-TR) and the folded
//                       median-prediction residual of every sample, as one
//                       32-bit token, laid out [wave group][sample][lane] so
//                       the coder's lanes read one coalesced line per sample;
//   ffv1_code_kernel    one lane per slice: put_symbol on the token stream.  The
//                       32 state bytes of the current context live in 8 VGPRs;
//                       the tokens are known in advance, so the state block of
//                       the sample two steps ahead is loaded while this one is
//                       coded (forwarded from registers when one of the two
//                       samples before it uses the same context).  A symbol's
//                       state bytes are all read before its first decision and
//                       written back after the last, so the LDS state-table
//                       lookups never sit on the range-coder chain.  The
//                       renormalisation only records `low >> 8` (+ one bit)
//                       per output byte: FFmpeg's outstanding-byte / carry
//                       logic is deferred to
//   ffv1_resolve_kernel one lane per slice: renorm_encoder's byte machine over
//                       those values -> the slice bytes and their CRC-32;
//   ffv1_pack_kernel    frame packets with their 8-byte slice footers.
// The coder is latency/issue-bound (dependent range updates, scattered state
// blocks), not HBM-bound: the figure of merit is frames/s (bench --workload ffv1).
#include <algorithm>
#include <cstring>
#include <memory>
#include <type_traits>
#include <vector>

#include "common.hpp"
#include "device.hpp"
#include "ffv1host.hpp"

namespace pp {

constexpr int kCtxSize = kFfv1CtxBytes;  // state bytes per context

// ---- device ---------------------------------------------------------------
struct Ffv1Args {
    const uint8_t *src[3];
    int64_t ls[3], fs[3];
    int w, h, bytes, bits, hsub, vsub, nh, nv, nslices;  // nslices = frames * nh * nv
    int64_t cap;            // per-slice output bytes (the 24-bit footer field bounds it)
    uint8_t *states;        // [nslices / 64][hot, cold][2 * nctx][64][16], primed to 128
    int64_t state_bytes;    // 2 * nctx * 32: one slice's luma and chroma context sets
    int nctx;               // contexts of the record's set (Ffv1Quant::contexts)
    int64_t *sizes;         // [nslices] coded bytes, -1 = overflow
    uint32_t *crcs;         // [nslices] CRC-32 of the coded bytes
    const uint8_t *tables;  // zero[256], one[256], crc table (1 KB)
    uint32_t *tok;          // [nslices / 64][tok_len][64] tokens
    int64_t tok_len;        // tokens per slice, max over the grid
    uint32_t *raw;          // [nslices][raw_cap] renorm records, two per dword; ffv1_resolve_kernel
                            // overwrites them in place with the slice bytes (bytes trail records)
    int64_t raw_cap;        // dwords per slice (this launch: the budget over its slices)
    int32_t *nraw;          // [nslices] records, -1 = overflow
    int lpw;                // slices (active lanes) per 64-lane coder workgroup
    int rlpw;               // the same for ffv1_resolve_kernel
    int debug;              // PIXPATH_FFV1_DEBUG (timing ablation only; the output is wrong):
                            // 1 no block loads, 2 no block stores, 4 no record flush
    int qthr[5];            // the record's quantiser (Ffv1Quant): thresholds, unused ones 1024
    int qL;                 // its levels: context = q(L - TL) + qL q(TL - T) + qL^2 q(T - TR)
};

// ffv1_quant (ffv1host.cpp) on the device: the number of thresholds <= |d|
__device__ inline int dquant(int d, const int (&thr)[5]) {  // d already & 0xFF
    const int m = d < 128 ? d : (d == 128 ? 127 : 256 - d);
    const int q = (m >= thr[0]) + (m >= thr[1]) + (m >= thr[2]) + (m >= thr[3]) + (m >= thr[4]);
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

// ---- slice geometry (RFC 9043 4.6: slice_x .. in units of the grid) ---------
struct SliceGeo {
    int frame, s, sx, sy, x0, x1, y0, y1, lw, lh, cw, ch;
    __device__ __host__ int len() const { return lw * lh + 2 * cw * ch; }
};
__device__ __host__ inline SliceGeo slice_geo(int g, int w, int h, int nh, int nv, int hsub, int vsub) {
    SliceGeo q;
    const int per = nh * nv;
    q.frame = g / per;
    q.s = g - q.frame * per;
    q.sy = q.s / nh;
    q.sx = q.s - q.sy * nh;
    q.x0 = (int)((int64_t)q.sx * w / nh);
    q.x1 = (int)((int64_t)(q.sx + 1) * w / nh);
    q.y0 = (int)((int64_t)q.sy * h / nv);
    q.y1 = (int)((int64_t)(q.sy + 1) * h / nv);
    q.lw = q.x1 - q.x0;
    q.lh = q.y1 - q.y0;
    q.cw = (q.lw + (1 << hsub) - 1) >> hsub;
    q.ch = (q.lh + (1 << vsub) - 1) >> vsub;
    return q;
}

// ---- 1. modelling: tokens (context key << 16 | folded residual) -------------
// One workgroup of 256 threads per (64-slice wave group, plane row).  A token
// depends only on input samples (L = cur[x-1], T / TL / TR from the row
// above; FFmpeg's borders at the slice edges), so every token is independent:
// the row and the row above of the 64 slices are staged in LDS kMX columns at
// a time (consecutive threads read consecutive samples of one slice row:
// coalesced), then thread (lane = t & 63, column phase = t >> 6) computes the
// tokens of its lane at columns phase, phase + 4, ... and the 64 threads of a
// wave store one token column as one contiguous 256-B line
// ([wave group][sample][lane], the coder's layout).  Lanes of one workgroup
// can be in different planes (slices of unequal height), so every row pointer
// and width is per lane.  key = plane set * nctx + |context|; the residual is
// negated with the context (encode_line), folded to the bit depth, int16.
constexpr int kMX = 64;          // columns per staged chunk
constexpr int kMS = kMX + 2;     // staged samples per row: x0 - 1 .. x0 + 64
constexpr int kMLane = 2 * kMS + 1;  // lane stride in LDS (odd: no bank conflicts)
template <typename ST>
__global__ __launch_bounds__(256) void ffv1_model_kernel(const Ffv1Args a) {
    __shared__ int s_row[64 * kMLane];        // [lane][top, cur][column x0 - 1 + j]
    __shared__ uint64_t s_ptr[64][2];         // [lane][row above, row]
    __shared__ int s_info[64][5];             // pw, has-T, TL0, token offset, context key base
    __shared__ int s_q[256];                  // quantiser level of d & 0xFF (ffv1_quant)
    const int t = threadIdx.x;
    const int wg = blockIdx.y;
    s_q[t] = dquant(t, a.qthr);
    if (t < 64) {
        const int g = wg * 64 + t;
        const bool live = g < a.nslices;
        const SliceGeo q = slice_geo(live ? g : 0, a.w, a.h, a.nh, a.nv, a.hsub, a.vsub);
        int r = blockIdx.x, p = 0, off = 0;
        bool on = live;
        if (r < q.lh) {
            p = 0;
        } else if ((r -= q.lh) < q.ch) {
            p = 1; off = q.lw * q.lh;
        } else if ((r -= q.ch) < q.ch) {
            p = 2; off = q.lw * q.lh + q.cw * q.ch;
        } else {
            on = false;
        }
        const int y = r;
        const int pw = on ? (p ? q.cw : q.lw) : 0;
        const int px0 = p ? q.x0 >> a.hsub : q.x0, py0 = p ? q.y0 >> a.vsub : q.y0;
        const uint8_t *src = p == 0 ? a.src[0] : p == 1 ? a.src[1] : a.src[2];
        const int64_t ls = p == 0 ? a.ls[0] : p == 1 ? a.ls[1] : a.ls[2];
        const int64_t fs = p == 0 ? a.fs[0] : p == 1 ? a.fs[1] : a.fs[2];
        const uint8_t *rowb = on ? src + q.frame * fs + (int64_t)(py0 + y) * ls + (int64_t)px0 * sizeof(ST) : src;
        s_ptr[t][0] = reinterpret_cast<uint64_t>(rowb - ls);
        s_ptr[t][1] = reinterpret_cast<uint64_t>(rowb);
        s_info[t][0] = pw;
        s_info[t][1] = on && y > 0;
        // FFmpeg's sample-buffer borders: 0 above the slice, L = T at column 0,
        // TL at column 0 = first sample two rows up, TR past the last column = T
        s_info[t][2] = on && y > 1 ? reinterpret_cast<const ST *>(rowb - 2 * ls)[0] : 0;
        s_info[t][3] = off + y * pw;
        s_info[t][4] = p ? a.nctx : 0;
    }
    __syncthreads();
    const int lane = t & 63, ph = t >> 6;
    const int pw = s_info[lane][0], TL0 = s_info[lane][2];
    const int mask = (1 << a.bits) - 1, half = 1 << (a.bits - 1);
    uint32_t *out = a.tok + ((int64_t)wg * a.tok_len + s_info[lane][3]) * 64 + lane;
    const uint32_t kbase = (uint32_t)s_info[lane][4];
    int pw_max = 0;
    for (int j = 0; j < 64; ++j) pw_max = max(pw_max, s_info[j][0]);
    int *const my = s_row + lane * kMLane;
    for (int x0 = 0; x0 < pw_max; x0 += kMX) {
        if (x0) __syncthreads();  // the previous chunk's LDS reads are done
        // stage columns x0 - 1 .. x0 + 64 of the row above and the row of every
        // lane (segment = lane j, row rw) as 16-byte pieces of the aligned span
        // x0 - SP .. x0 + 64 + SP (SP samples per piece: x0 is a multiple of
        // 64, so every piece of a 16-byte aligned row is 16-byte aligned --
        // 8-bit pieces started 8 bytes off): thread t takes pieces t, t + 256, ... of the
        // chunk, so consecutive threads read consecutive bytes of one slice row
        // (a per-thread walk of 2-byte loads, one row per lane, was bound by
        // the L1 -> L2 requests: 3.3e9 per 600 frames, profiles/r5/ffv1_pmc.txt).
        // A piece past the row's ends, or of a row not 16-byte aligned, is read
        // sample by sample with the bounds check (zeros outside the row).
        {
            constexpr int SP = 16 / (int)sizeof(ST);  // samples per piece
            constexpr int NP = (kMX + 2 * SP) / SP;   // pieces per segment
            for (int i = t; i < 128 * NP; i += 256) {
                const int seg = i / NP, pc = i - seg * NP, j = seg >> 1, rw = seg & 1;
                const ST *rp = reinterpret_cast<const ST *>(s_ptr[j][rw]);
                const int lim = (rw || s_info[j][1]) ? s_info[j][0] : 0;  // row above absent: zeros
                const int s0 = x0 - SP + pc * SP;
                int *dst = s_row + j * kMLane + rw * kMS + (s0 - (x0 - 1));  // column of sample s0
                ST v[SP];
                if (s0 >= 0 && s0 + SP <= lim && (reinterpret_cast<uintptr_t>(rp) & 15) == 0) {
                    const uint4 q = *reinterpret_cast<const uint4 *>(rp + s0);
                    __builtin_memcpy(v, &q, 16);
                } else {
#pragma unroll
                    for (int e = 0; e < SP; ++e) v[e] = (s0 + e >= 0 && s0 + e < lim) ? rp[s0 + e] : (ST)0;
                }
#pragma unroll
                for (int e = 0; e < SP; ++e) {
                    const int col = s0 - (x0 - 1) + e;
                    if (col >= 0 && col < kMS) dst[e] = (int)v[e];
                }
            }
        }
        __syncthreads();
        const int xe = min(pw, x0 + kMX);
        for (int x = x0 + ph; x < xe; x += 4) {
            const int c = x - x0 + 1;
            const int T = my[c], v = my[kMS + c];
            const int L = x ? my[kMS + c - 1] : T;
            const int TL = x ? my[c - 1] : TL0;
            const int TR = x + 1 < pw ? my[c + 1] : T;
            int ctx = s_q[(L - TL) & 0xFF] + a.qL * (s_q[(TL - T) & 0xFF] + a.qL * s_q[(T - TR) & 0xFF]);
            int diff = v - median3(L, L + T - TL, T);
            if (ctx < 0) {
                ctx = -ctx;
                diff = -diff;
            }
            diff &= mask;
            diff = diff >= half ? diff - (mask + 1) : diff;
            out[(int64_t)x * 64] = ((kbase + (uint32_t)ctx) << 16) | ((uint32_t)diff & 0xFFFFu);
        }
    }
}

// ---- 2. coding ---------------------------------------------------------------
// The range coder of one lane.  A lane's decisions are the wave's work unit:
// the 64 lanes of a wave code different slices, so a symbol costs the wave the
// LONGEST symbol among its lanes.  Every decision is therefore branch-free
// (a lane whose symbol is shorter codes no-op decisions: state 0, bit 0 leaves
// low / range unchanged), and the wave-uniform exponent bound E (four ballots)
// skips the decision slots no lane needs with scalar branches.
// Renormalisation records `low` (before the shift) per output byte in the
// lane's LDS ring with an unconditional store at the write position (a
// decision that does not renormalise leaves the position, so the next one
// overwrites it); the ring leaves kFlush records per 4 samples, packed to 16 bits
// ((low >> 8) | ((low & 0xFF) == 0) << 9), and ffv1_resolve_kernel turns them
// into bytes exactly as renorm_encoder does.  The 4 unrolled coding steps
// issue a fixed pattern of vector-memory operations (token load, block load,
// block store per step, the record store in the fourth), so the wait for a
// block loaded two steps earlier can leave the younger loads and stores in
// flight (vmcnt counts both, in order).
constexpr int kRing = 128;   // records per lane ring (LDS, u32)
// lane stride of the rings: odd, so the 64 lanes' stores at similar write
// positions fall in different LDS banks (a 128-dword stride put every lane's
// record store of a decision in the same bank: a 64-way conflict per decision)
constexpr int kRingStride = kRing + 1;
constexpr int kFlush = 8;    // records stored per flush (16 B), one flush per 4 samples (~2.4 records on
                             // compressible content, ~5.6 on 10-bit noise: the ring only fills on longer bursts)
struct Enc {
    uint32_t low, range;
    uint32_t *ring;          // this lane's kRing records
    uint32_t wp;             // records pushed
};

// one binary decision (put_rac) with state value s, branch-free; s = 0 and
// bit = 0 is a no-op (r1 = 0: low and range stay, range >= 0x100: no renorm)
__device__ __forceinline__ void enc_dec(Enc &c, uint32_t s, bool bit) {
    const uint32_t r1 = __umul24(c.range, s) >> 8;
    const uint32_t rz = c.range - r1;
    c.low += bit ? rz : 0u;
    c.range = bit ? r1 : rz;
    c.ring[c.wp & (kRing - 1)] = c.low;
    const bool rn = c.range < 0x100u;
    c.wp += rn ? 1u : 0u;
    c.low = rn ? (c.low << 8) & 0xFF00u : c.low;
    c.range = rn ? c.range << 8 : c.range;
}

// renorm_encoder for the terminating flushes (outside the hot loop)
__device__ __forceinline__ void enc_renorm(Enc &c) {
    if (c.range < 0x100u) {
        c.ring[c.wp & (kRing - 1)] = c.low;
        ++c.wp;
        c.low = (c.low & 0xFFu) << 8;
        c.range <<= 8;
    }
}

// state byte k of a 32-byte block held in 8 dwords (k a compile-time constant
// after unrolling: no dynamic register indexing)
__device__ __forceinline__ uint32_t sget(const uint32_t (&b)[8], int k) { return (b[k >> 2] >> ((k & 3) * 8)) & 0xFFu; }
__device__ __forceinline__ void sput(uint32_t (&b)[8], int k, uint32_t v) {
    b[k >> 2] = (b[k >> 2] & ~(0xFFu << ((k & 3) * 8))) | (v << ((k & 3) * 8));
}
// runtime index k in 8..23 (the sign state 11 + e), branch-free selects
__device__ __forceinline__ uint32_t sget_dyn(const uint32_t (&b)[8], int k) {
    const int w = k >> 2;
    const uint32_t lo = (w & 1) ? b[3] : b[2], hi = (w & 1) ? b[5] : b[4];
    return __builtin_amdgcn_ubfe(w >= 4 ? hi : lo, (k & 3) * 8, 8);
}
__device__ __forceinline__ void sput_dyn(uint32_t (&b)[8], int k, uint32_t v, bool on) {
    const int w = k >> 2;
    const uint32_t sh = (k & 3) * 8, m = ~(0xFFu << sh), nv = v << sh;
    b[2] = on && w == 2 ? (b[2] & m) | nv : b[2];
    b[3] = on && w == 3 ? (b[3] & m) | nv : b[3];
    b[4] = on && w == 4 ? (b[4] & m) | nv : b[4];
    b[5] = on && w == 5 ? (b[5] & m) | nv : b[5];
}

// wave-uniform max of e over the live lanes (e in -1..15): a binary search of ballots
__device__ __forceinline__ int wave_max_e(int e) {
    int E = -1;
    if (__builtin_amdgcn_ballot_w64(e >= E + 8)) E += 8;
    if (__builtin_amdgcn_ballot_w64(e >= E + 4)) E += 4;
    if (__builtin_amdgcn_ballot_w64(e >= E + 2)) E += 2;
    if (__builtin_amdgcn_ballot_w64(e >= E + 1)) E += 1;
    return __builtin_amdgcn_readfirstlane(E);
}

// put_symbol (ffv1enc.c put_symbol_inline) on a register block, |v| < 1024:
// every state byte the symbol uses is read from `b` before the first decision
// (each is used at most once per symbol), the next states come from the LDS
// tables in one batch of reads (they depend on the bits only, not on low /
// range), and the updated bytes are written after the last decision.
template <bool SIGNED>
__device__ __forceinline__ void enc_symbol(Enc &c, uint32_t (&b)[8], int v, const uint8_t *tab) {
    const uint32_t a = (uint32_t)(v < 0 ? -v : v);
    const bool nz = v != 0;
    const int e = nz ? 31 - __clz(a) : -1;
    const int E = wave_max_e(e);
    const uint32_t s0 = sget(b, 0);
    uint32_t su[10], sm[9], ss = 0, n0, nu[10], nm[9], nsg = 0;
    n0 = tab[s0 | (nz ? 0u : 256u)];
#pragma unroll
    for (int i = 0; i < 10; ++i)
        if (i <= E) {
            su[i] = sget(b, 1 + i);
            nu[i] = tab[su[i] | (i < e ? 256u : 0u)];
        }
#pragma unroll
    for (int i = 0; i < 9; ++i)
        if (i < E) {
            sm[i] = sget(b, 22 + i);
            nm[i] = tab[sm[i] | (((a >> i) & 1u) << 8)];
        }
    if (SIGNED && E >= 0) {
        ss = sget_dyn(b, 11 + (e < 0 ? 0 : e));
        nsg = tab[ss | (v < 0 ? 256u : 0u)];
    }
    enc_dec(c, s0, !nz);
#pragma unroll
    for (int i = 0; i < 10; ++i)
        if (i <= E) enc_dec(c, i <= e ? su[i] : 0u, i < e);
#pragma unroll
    for (int i = 8; i >= 0; --i)
        if (i < E) enc_dec(c, i < e ? sm[i] : 0u, i < e && ((a >> i) & 1u));
    if (SIGNED && E >= 0) enc_dec(c, nz ? ss : 0u, v < 0);
    sput(b, 0, n0);
#pragma unroll
    for (int i = 0; i < 10; ++i)
        if (i <= E) sput(b, 1 + i, i <= e ? nu[i] : su[i]);
#pragma unroll
    for (int i = 0; i < 9; ++i)
        if (i < E) sput(b, 22 + i, i < e ? nm[i] : sm[i]);
    if (SIGNED && E >= 0) sput_dyn(b, 11 + (e < 0 ? 0 : e), nsg, nz);
}

// A context's 32 state bytes split in two 16-byte halves (the decoder's
// layout, ffv1dec.hip).  HOT, the block the coder forwards and prefetches:
// [0] zero flag, [1..5] exponent bits 0..4, [6..10] sign for e = 0..4,
// [11..14] mantissa bits 0..3 -- every state a residual below 32 touches.
// COLD, read and written in place only while the wave's longest exponent is
// >= 5: [0..4] exponent bits 5..9, [5..9] sign for e = 5..9, [10..14]
// mantissa bits 4..8.
__device__ __forceinline__ uint32_t hget(const uint32_t (&b)[4], int k) { return (b[k >> 2] >> ((k & 3) * 8)) & 0xFFu; }
__device__ __forceinline__ void hput(uint32_t (&b)[4], int k, uint32_t v) {
    b[k >> 2] = (b[k >> 2] & ~(0xFFu << ((k & 3) * 8))) | (v << ((k & 3) * 8));
}
// enc_symbol on the split block: the same decisions in the same order
template <bool SIGNED>
__device__ __forceinline__ void enc_symbol_split(Enc &c, uint32_t (&b)[4], uint8_t *cold, int v, const uint8_t *tab) {
    const uint32_t a = (uint32_t)(v < 0 ? -v : v);
    const bool nz = v != 0;
    const int e = nz ? 31 - __clz(a) : -1;
    const int E = wave_max_e(e);
    uint32_t cb[4] = {0u, 0u, 0u, 0u};
    if (E >= 5) {  // wave-uniform
        const uint4 x = *reinterpret_cast<const uint4 *>(cold);
        cb[0] = x.x; cb[1] = x.y; cb[2] = x.z; cb[3] = x.w;
    }
    const uint32_t s0 = hget(b, 0);
    uint32_t su[10], sm[9], ss = 0, n0, nu[10], nm[9], nsg = 0;
    n0 = tab[s0 | (nz ? 0u : 256u)];
#pragma unroll
    for (int i = 0; i < 10; ++i)
        if (i <= E) {
            su[i] = i < 5 ? hget(b, 1 + i) : hget(cb, i - 5);
            nu[i] = tab[su[i] | (i < e ? 256u : 0u)];
        }
#pragma unroll
    for (int i = 0; i < 9; ++i)
        if (i < E) {
            sm[i] = i < 4 ? hget(b, 11 + i) : hget(cb, 10 + i - 4);
            nm[i] = tab[sm[i] | (((a >> i) & 1u) << 8)];
        }
    const int es = e < 0 ? 0 : e;
    if (SIGNED && E >= 0) {  // sign state of exponent es: compile-time byte indices under selects
#pragma unroll
        for (int i = 0; i < 10; ++i) ss = es == i ? (i < 5 ? hget(b, 6 + i) : hget(cb, i)) : ss;
        nsg = tab[ss | (v < 0 ? 256u : 0u)];
    }
    enc_dec(c, s0, !nz);
#pragma unroll
    for (int i = 0; i < 10; ++i)
        if (i <= E) enc_dec(c, i <= e ? su[i] : 0u, i < e);
#pragma unroll
    for (int i = 8; i >= 0; --i)
        if (i < E) enc_dec(c, i < e ? sm[i] : 0u, i < e && ((a >> i) & 1u));
    if (SIGNED && E >= 0) enc_dec(c, nz ? ss : 0u, v < 0);
    hput(b, 0, n0);
#pragma unroll
    for (int i = 0; i < 10; ++i)
        if (i <= E) {
            if (i < 5) hput(b, 1 + i, i <= e ? nu[i] : su[i]);
            else hput(cb, i - 5, i <= e ? nu[i] : su[i]);
        }
#pragma unroll
    for (int i = 0; i < 9; ++i)
        if (i < E) {
            if (i < 4) hput(b, 11 + i, i < e ? nm[i] : sm[i]);
            else hput(cb, 10 + i - 4, i < e ? nm[i] : sm[i]);
        }
    if (SIGNED && E >= 0) {
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            const bool on = nz && es == i;
            if (i < 5) hput(b, 6 + i, on ? nsg : hget(b, 6 + i));
            else hput(cb, i, on ? nsg : hget(cb, i));
        }
    }
    if (E >= 5) *reinterpret_cast<uint4 *>(cold) = make_uint4(cb[0], cb[1], cb[2], cb[3]);
}

__device__ __forceinline__ void hblk_load(uint32_t (&b)[4], const uint8_t *p) {
    const uint4 x = *reinterpret_cast<const uint4 *>(p);
    b[0] = x.x; b[1] = x.y; b[2] = x.z; b[3] = x.w;
}
__device__ __forceinline__ void hblk_store(uint8_t *p, const uint32_t (&b)[4]) {
    *reinterpret_cast<uint4 *>(p) = make_uint4(b[0], b[1], b[2], b[3]);
}
__device__ __forceinline__ void hblk_sel(uint32_t (&d)[4], bool c, const uint32_t (&x)[4], const uint32_t (&y)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = c ? x[i] : y[i];
}

__device__ __forceinline__ void blk_load(uint32_t (&b)[8], const uint8_t *p) {
    const uint4 x = reinterpret_cast<const uint4 *>(p)[0], y = reinterpret_cast<const uint4 *>(p)[1];
    b[0] = x.x; b[1] = x.y; b[2] = x.z; b[3] = x.w; b[4] = y.x; b[5] = y.y; b[6] = y.z; b[7] = y.w;
}
__device__ __forceinline__ void blk_store(uint8_t *p, const uint32_t (&b)[8]) {
    reinterpret_cast<uint4 *>(p)[0] = make_uint4(b[0], b[1], b[2], b[3]);
    reinterpret_cast<uint4 *>(p)[1] = make_uint4(b[4], b[5], b[6], b[7]);
}
__device__ __forceinline__ void blk_sel(uint32_t (&d)[8], bool c, const uint32_t (&x)[8], const uint32_t (&y)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = c ? x[i] : y[i];
}

// 16-bit renorm record of a recorded `low`: low >> 8 (9 bits) | exact << 9
__device__ __forceinline__ uint32_t rec16(uint32_t low) { return (low >> 8) | ((low & 0xFFu) == 0u ? 0x200u : 0u); }

__global__ __launch_bounds__(64) void ffv1_code_kernel(const Ffv1Args a) {
    __shared__ uint8_t s_tab[512];  // zero[256], one[256]
    __shared__ __align__(16) uint32_t s_ring[64 * kRingStride];
    for (int i = threadIdx.x; i < 512; i += 64) s_tab[i] = a.tables[i];
    __syncthreads();
    const int lane = threadIdx.x;
    if (lane >= a.lpw) return;
    const int g = blockIdx.x * a.lpw + lane;
    if (g >= a.nslices) return;
    const SliceGeo q = slice_geo(g, a.w, a.h, a.nh, a.nv, a.hsub, a.vsub);
    const int len = q.len();
    // context states of the 64-slice group interleaved by slice, hot halves
    // then cold halves: context k of slice g at [g / 64][half][k][g % 64][16]
    // -- a 128-B line holds one context's half of 8 slices (a context that is
    // hot in one slice is hot in its neighbours)
    uint8_t *const st0 = a.states + (int64_t)(g >> 6) * (64 * a.state_bytes) + (g & 63) * 16;
    uint8_t *const co0 = st0 + 64 * a.state_bytes / 2;
    constexpr int kCtxStride = 64 * 16;
    // tokens of slice g: group g / 64 of the modelling layout, lane g % 64
    const uint32_t *tp = a.tok + (int64_t)(g >> 6) * a.tok_len * 64 + (g & 63);
    Enc c;
    c.low = 0; c.range = 0xFF00; c.wp = 0;
    c.ring = s_ring + lane * kRingStride;
    // records leave the ring kFlush at a time (packed to 16 bits) into the
    // lane's record buffer; `fp` records are final there, the rest of the
    // kFlush is rewritten next step
    uint16_t *const out = reinterpret_cast<uint16_t *>(a.raw + (int64_t)g * a.raw_cap);
    const uint32_t cap = (uint32_t)(a.raw_cap * 2) & ~(uint32_t)(kFlush - 1);  // records the buffer holds
    uint32_t fp = 0;
    bool over = false;
    auto flush = [&]() {
        const uint32_t *r = c.ring + (fp & (kRing - 1));  // dword reads (the lane stride is odd)
        uint4 pk;
        pk.x = rec16(r[0]) | (rec16(r[1]) << 16);
        pk.y = rec16(r[2]) | (rec16(r[3]) << 16);
        pk.z = rec16(r[4]) | (rec16(r[5]) << 16);
        pk.w = rec16(r[6]) | (rec16(r[7]) << 16);
        *reinterpret_cast<uint4 *>(out + (fp < cap ? fp : cap - kFlush)) = pk;
        // exact: a store at the write position (renormalising or not) reaches
        // the oldest unflushed record only once kRing records are pending, and
        // the pending count only grows between flushes
        over |= c.wp - fp >= (uint32_t)kRing || fp >= cap;
        if (c.wp - fp >= (uint32_t)kFlush) fp += kFlush;
    };
    // keyframe bit (first slice of a frame), then the slice header with its own 32 states:
    // slice x, y, width - 1, height - 1 (slice units), table set of Y and of Cb/Cr,
    // picture_structure 3 (progressive), SAR 1:1 (setsar=1/1)
    if (q.s == 0) enc_dec(c, 128, true);
    {
        uint32_t hb[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) hb[i] = 0x80808080u;
        const int hv[9] = {q.sx, q.sy, 0, 0, 0, 0, 3, 1, 1};
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            enc_symbol<false>(c, hb, hv[i], s_tab);
            flush();
        }
    }
    // token stream with block forwarding (see the file comment); every step
    // issues the same vector-memory operations: one token load, one block
    // load, one block store, one ring flush
    // (an unconditional load: past the end it rereads the last token, a valid key)
    auto tok = [&](int i) { return tp[(int64_t)min(i, len - 1) * 64]; };
    // tokens and prefetched blocks live in fixed registers (a ring indexed by
    // the step's phase, 4x unrolled): a register copy of an in-flight load
    // would make the compiler wait for it at the copy.  (A 4-sample block
    // prefetch with forwarding from the last 4 samples measured the same
    // 161-165 ms per 600 frames: the compiler rotates the longer rings
    // through register copies at the loop latch and waits there.)
    uint32_t tk[4] = {tok(0), tok(1), tok(2), tok(3)};
    int km2 = -1, km1 = -1;
    uint32_t cur[4], prev[4], pre[2][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) cur[i] = prev[i] = 0u;
    hblk_load(pre[0], st0 + (tk[0] >> 16) * kCtxStride);
    hblk_load(pre[1], st0 + (tk[1] >> 16) * kCtxStride);
    auto step = [&](int i, auto ph_c) {
        constexpr int PH = decltype(ph_c)::value;
        const uint32_t t0 = tk[PH], t2 = tk[(PH + 2) & 3];
        const int k0 = (int)(t0 >> 16);
        const int v = (int)(int16_t)(t0 & 0xFFFFu);
        uint32_t b[4];
        // hot block of this sample: the previous sample's, the one before, or the prefetched
        {
            uint32_t tmp[4];
            hblk_sel(tmp, k0 == km2, prev, pre[PH & 1]);
            hblk_sel(b, k0 == km1, cur, tmp);
        }
        // the hot block of sample i + 2 (used unless sample i or i + 1 forwards it)
        if (!(PP_ABLATE(a.debug) & 1)) hblk_load(pre[PH & 1], st0 + (t2 >> 16) * kCtxStride);
        tk[PH] = tok(i + 4);
        enc_symbol_split<true>(c, b, co0 + k0 * kCtxStride, v, s_tab);
        if (!(PP_ABLATE(a.debug) & 2)) hblk_store(st0 + k0 * kCtxStride, b);
        if (PH == 3 && !(PP_ABLATE(a.debug) & 4)) flush();
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            prev[j] = cur[j];
            cur[j] = b[j];
        }
        km2 = km1;
        km1 = k0;
    };
    int i = 0;
    for (; i + 3 < len; i += 4) {
        step(i, std::integral_constant<int, 0>{});
        step(i + 1, std::integral_constant<int, 1>{});
        step(i + 2, std::integral_constant<int, 2>{});
        step(i + 3, std::integral_constant<int, 3>{});
    }
    if (i < len) step(i, std::integral_constant<int, 0>{});
    if (i + 1 < len) step(i + 1, std::integral_constant<int, 1>{});
    if (i + 2 < len) step(i + 2, std::integral_constant<int, 2>{});
    flush();
    // closing 0 bit at state 129 (ffv1enc.c encode_frame), ff_rac_terminate's two flushes
    enc_dec(c, 129, false);
    c.range = 0xFF;
    c.low += 0xFF;
    enc_renorm(c);
    c.range = 0xFF;
    enc_renorm(c);
    while (fp < c.wp) {
        flush();
        if (c.wp - fp < (uint32_t)kFlush) {  // the partial tail is stored; done
            flush();
            break;
        }
    }
    a.nraw[g] = over || c.wp > cap ? -1 : (int32_t)c.wp;
}

// ---- 3. bytes: renorm_encoder's outstanding-byte machine ----------------------
__global__ __launch_bounds__(64) void ffv1_resolve_kernel(const Ffv1Args a) {
    // slice-by-4 CRC tables: s_crc[k][i] = the byte table advanced by k zero
    // bytes, so a whole output word updates the CRC with 4 independent lookups
    // (one LDS latency on the chain per 4 bytes instead of per byte)
    __shared__ uint32_t s_crc[4][256];
    for (int i = threadIdx.x; i < 256; i += 64) s_crc[0][i] = reinterpret_cast<const uint32_t *>(a.tables + 512)[i];
    __syncthreads();
    for (int k = 1; k < 4; ++k) {
        for (int i = threadIdx.x; i < 256; i += 64) {
            const uint32_t p = s_crc[k - 1][i];
            s_crc[k][i] = (p << 8) ^ s_crc[0][p >> 24];
        }
        __syncthreads();
    }
    if ((int)threadIdx.x >= a.rlpw) return;
    const int g = blockIdx.x * a.rlpw + threadIdx.x;
    if (g >= a.nslices) return;
    const int nraw = a.nraw[g];
    if (nraw < 0) {
        a.sizes[g] = -1;
        return;
    }
    // the slice bytes go over the slice's own records: byte k is emitted only
    // after record k + 1 (record r sits at bytes 2r, 2r + 1), and the blocks
    // in flight are ahead of both, so a word is written only where the records
    // have already been read
    const uint32_t *raw = a.raw + (int64_t)g * a.raw_cap;
    uint32_t *dst = a.raw + (int64_t)g * a.raw_cap;
    const int64_t capw = a.raw_cap;
    int64_t nb = 0;  // bytes emitted
    uint32_t word = 0, crc = 0;
    bool over = false;
    auto emit = [&](uint32_t v) {
        v &= 0xFFu;
        word |= v << ((nb & 3) * 8);
        if ((nb & 3) == 3) {  // bytes b0..b3 = word's bytes 0..3, b0 first
            crc = s_crc[3][(crc >> 24) ^ (word & 0xFFu)] ^ s_crc[2][((crc >> 16) & 0xFFu) ^ ((word >> 8) & 0xFFu)] ^
                  s_crc[1][((crc >> 8) & 0xFFu) ^ ((word >> 16) & 0xFFu)] ^ s_crc[0][(crc & 0xFFu) ^ (word >> 24)];
            if ((nb >> 2) < capw) dst[nb >> 2] = word;
            else over = true;
            word = 0;
        }
        ++nb;
    };
    int ob = -1, oc = 0;
    auto record = [&](uint32_t r) {
        const int hi = (int)(r & 0x1FFu);
        const bool exact = (r >> 9) & 1u;
        if (ob < 0) {
            ob = hi;
        } else if (hi < 0xFF || (hi == 0xFF && exact)) {  // low <= 0xFF00
            emit((uint32_t)ob);
            for (; oc; --oc) emit(0xFFu);
            ob = hi;
        } else if (hi >= 0x100) {  // low >= 0x10000: carry
            emit((uint32_t)ob + 1u);
            for (; oc; --oc) emit(0x00u);
            ob = hi - 0x100;
        } else {
            ++oc;
        }
    };
    // records 8 at a time (16 B), the blocks two ahead in flight: a record
    // load per pair of records used to put the memory latency on the chain
    const uint4 *rp = reinterpret_cast<const uint4 *>(raw);  // 16-B aligned (raw_cap % 4 == 0)
    const int nblk = (nraw + 7) >> 3;
    auto blk = [&](int b) { return rp[min(b, nblk - 1)]; };  // past the end: rereads the last block
    uint4 q[2] = {nblk > 0 ? blk(0) : make_uint4(0, 0, 0, 0), nblk > 1 ? blk(1) : make_uint4(0, 0, 0, 0)};
    auto block = [&](int b, uint4 &slot) {
        const uint4 v = slot;
        slot = blk(b + 2);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        const int m = min(8, nraw - 8 * b);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (k >= m) break;
            record((k & 1) ? w[k >> 1] >> 16 : w[k >> 1] & 0xFFFFu);
        }
    };
    for (int b = 0; b < nblk; b += 2) {
        block(b, q[0]);
        if (b + 1 < nblk) block(b + 1, q[1]);
    }
    if (nb & 3) {
        for (int64_t i = 0; i < (nb & 3); ++i)  // the last partial word, byte by byte
            crc = (crc << 8) ^ s_crc[0][(crc >> 24) ^ ((word >> (8 * i)) & 0xFFu)];
        if ((nb >> 2) < capw) dst[nb >> 2] = word;
        else over = true;
    }
    a.sizes[g] = over || nb + 8 > a.cap || nb > capw * 4 ? -1 : nb;
    a.crcs[g] = crc;
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
    int64_t cap = 0;           // per-slice output bytes (worst case, < 2^24)
    int64_t full_raw = 0;      // record dwords per slice for that worst case
    int64_t budget = 0;        // record dwords of the whole `raw` allocation
    int64_t tok_len = 0, rows_max = 0;
    uint8_t *states = nullptr, *tables = nullptr;
    int64_t *sizes = nullptr, *off = nullptr;
    uint32_t *crcs = nullptr, *tok = nullptr, *raw = nullptr;
    int32_t *nraw = nullptr;
    uint8_t *pk = nullptr;     // frame packets of the last encode, back to back
    int64_t pk_cap = 0, pk_len = 0;
    int launches = 0;          // launches of the last encode (> 1: a batch was split)
    Ffv1Quant quant;           // the record's 3-input quantiser
    int64_t state_bytes() const { return (int64_t)2 * quant.contexts() * kCtxSize; }
    std::vector<uint8_t> extradata;
};

// Record budget.  A slice's records (one 16-bit record per output byte) are
// sized per LAUNCH: the encoder holds `budget` dwords for all of them, and a
// launch of m frames gives each slice budget / (slices * m).  The default
// budget holds a full batch at half the raw sample bytes per slice (FFV1 codes
// video content at 2-4:1); a launch in which some slice runs out is re-coded
// as two launches of half the frames (twice the records per slice), down to
// the worst case (uniform noise: ~1.1x the raw bytes), so the output never
// depends on the budget.  Tokens stay sized for the whole batch.
constexpr int kBudgetDiv = 3;  // budget per slice = worst case / 3 (~0.5x the raw sample bytes)

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
    // every chroma sample in some slice: a slice at x0 covers chroma columns
    // [x0 >> hsub, +ceil((x1 - x0) / 2^hsub)) (RFC 9043 slice geometry), so an
    // odd boundary can leave the last chroma column / row in no slice -- e.g.
    // 333x191 4:2:0 in 3x3 slices; FFmpeg's encoder picks other grids
    // (ff_need_new_slices), this one refuses instead of dropping samples
    auto covers = [](int n, int ns, int sub) {
        int end = 0;
        for (int i = 0; i < ns; ++i) {
            const int a = (int)((int64_t)i * n / ns), b = (int)((int64_t)(i + 1) * n / ns);
            if ((a >> sub) > end) return false;
            end = std::max(end, (a >> sub) + (((b - a) + (1 << sub) - 1) >> sub));
        }
        return end >= ((n + (1 << sub) - 1) >> sub);
    };
    if (!covers(w, slices_h, fi.hsub) || !covers(h, slices_v, fi.vsub))
        PP_FAIL(PP_ERR_UNSUPPORTED, "slice grid %dx%d leaves chroma samples of a %dx%d frame in no slice", slices_h,
                slices_v, w, h);
    std::unique_ptr<pp_ffv1_enc> E(new pp_ffv1_enc());
    E->ctx = ctx; E->fmt = fmt; E->w = w; E->h = h; E->nh = slices_h; E->nv = slices_v; E->fi = fi;
    E->max_frames = max_frames;
    E->quant = ffv1_default_quant(fi.depth);
    // configuration record (RFC 9043 4.2, ffv1enc.c write_extradata; ffv1host.cpp)
    if (const char *e = PP_KNOB("PIXPATH_FFV1_QBOUNDS")) {  // measurement build: the quantiser's thresholds
        Ffv1Quant q;
        q.n = 0;
        for (const char *c = e; *c && q.n < 5;) {
            const int v = std::atoi(c);
            if (v < 1 || v > 127 || (q.n && v <= q.thr[q.n - 1])) PP_FAIL(PP_ERR_INVALID, "PIXPATH_FFV1_QBOUNDS %s", e);
            q.thr[q.n++] = v;
            while (*c && *c != ',') ++c;
            if (*c == ',') ++c;
        }
        if (!q.n) PP_FAIL(PP_ERR_INVALID, "PIXPATH_FFV1_QBOUNDS %s", e);
        E->quant = q;
    }
    E->extradata = ffv1_write_record(fi.depth, fi.hsub, fi.vsub, slices_h, slices_v, E->quant);
    if (!ctx) {  // host-only: configuration record only
        *out = E.release();
        return PP_OK;
    }
    const int per = slices_h * slices_v;
    const int64_t ns = (int64_t)per * max_frames;
    const int64_t ns64 = (ns + 63) / 64 * 64;
    const int bytes = fi.depth > 8 ? 2 : 1;
    // the largest slice of the grid (slices differ by one column / row at most)
    int64_t len_max = 0, rows = 0;
    for (int s = 0; s < per; ++s) {
        const SliceGeo q = slice_geo(s, w, h, slices_h, slices_v, fi.hsub, fi.vsub);
        len_max = std::max<int64_t>(len_max, q.len());
        rows = std::max<int64_t>(rows, q.lh + 2 * q.ch);
    }
    E->tok_len = len_max;
    E->rows_max = rows;
    const int64_t raw = len_max * bytes;
    // worst case (uniform noise) codes ~1.1x the raw samples; a slice larger
    // than the 24-bit footer size field (FFmpeg asserts < 1 << 24) is refused
    E->cap = ((raw * 3 / 2 + 4096) + 255) & ~int64_t(255);
    E->cap = std::min<int64_t>(E->cap, ((int64_t)1 << 24) - 256);
    E->full_raw = (E->cap / 2 + 4 + 3) & ~int64_t(3);  // two records (one per output byte) per dword, 16-B rows
    // every slice of one frame at the worst case always fits (the last split)
    E->budget = std::max<int64_t>(ns * (E->full_raw / kBudgetDiv), (int64_t)per * E->full_raw);
    PP_HIP(hipSetDevice(ctx->device));
    PP_HIP(hipMalloc(&E->states, (size_t)E->state_bytes() * ns64));
    PP_HIP(hipMalloc(&E->sizes, sizeof(int64_t) * ns));
    PP_HIP(hipMalloc(&E->off, sizeof(int64_t) * ns));
    PP_HIP(hipMalloc(&E->crcs, sizeof(uint32_t) * ns));
    PP_HIP(hipMalloc(&E->tok, sizeof(uint32_t) * (size_t)(ns64 * len_max)));
    PP_HIP(hipMalloc(&E->raw, sizeof(uint32_t) * (size_t)E->budget));
    PP_HIP(hipMalloc(&E->nraw, sizeof(int32_t) * ns));
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
    for (void *p : {(void *)E->states, (void *)E->sizes, (void *)E->off, (void *)E->crcs, (void *)E->tables,
                    (void *)E->tok, (void *)E->raw, (void *)E->nraw, (void *)E->pk})
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

extern "C" int pp_ffv1_encoder_memory(const pp_ffv1_enc *E, int64_t *bytes) {
    if (!E || !bytes) PP_FAIL(PP_ERR_INVALID, "null argument");
    const int64_t ns = (int64_t)E->nh * E->nv * E->max_frames, ns64 = (ns + 63) / 64 * 64;
    *bytes = E->ctx ? E->state_bytes() * ns64 + (8 + 8 + 4 + 4) * ns + 4 * ns64 * E->tok_len + 4 * E->budget +
                          1536 + E->pk_cap
                    : 0;
    return PP_OK;
}

// Grow the packet buffer to `need` bytes keeping its first `keep` bytes.
static int pk_reserve(pp_ffv1_enc *E, int64_t need, int64_t keep, hipStream_t st) {
    if (need <= E->pk_cap) return PP_OK;
    const int64_t cap = std::max<int64_t>(need, E->pk_cap + E->pk_cap / 2);
    uint8_t *p = nullptr;
    PP_HIP(hipMalloc(&p, cap));
    if (keep) {
        if (hipMemcpyAsync(p, E->pk, keep, hipMemcpyDeviceToDevice, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) {
            (void)hipFree(p);
            PP_FAIL(PP_ERR_HIP, "packet buffer copy failed");
        }
    }
    if (E->pk) PP_HIP(hipFree(E->pk));
    E->pk = p;
    E->pk_cap = cap;
    return PP_OK;
}

extern "C" int64_t pp_ffv1_encode_packets(pp_ffv1_enc *E, const pp_frames *src, int nframes, int64_t *frame_sizes,
                                          const uint8_t **packets, void *stream) {
    if (!E || !src || !frame_sizes || nframes < 0) PP_FAIL(PP_ERR_INVALID, "null argument");
    if (!E->ctx) PP_FAIL(PP_ERR_INVALID, "host-only encoder cannot encode");
    if (nframes > E->max_frames) PP_FAIL(PP_ERR_INVALID, "%d frames > max_frames %d", nframes, E->max_frames);
    if (packets) *packets = nullptr;
    E->pk_len = 0;
    E->launches = 0;
    if (nframes == 0) return 0;
    hipStream_t st = static_cast<hipStream_t>(stream);
    PP_HIP(hipSetDevice(E->ctx->device));
    const int per = E->nh * E->nv;
    int64_t total = 0;
    int f0 = 0, m = nframes;
    std::vector<int64_t> sizes, off;
    while (f0 < nframes) {
        m = std::min(m, nframes - f0);
        const int ns = per * m;
        // records per slice for this launch: the budget over its slices, at most the worst case
        const int64_t rcap = std::min<int64_t>(E->full_raw, E->budget / ns / 4 * 4);
        Ffv1Args a{};
        for (int p = 0; p < 3; ++p) {
            a.src[p] = static_cast<const uint8_t *>(src->data[p]) + (int64_t)f0 * src->frame_stride[p];
            a.ls[p] = src->linesize[p];
            a.fs[p] = src->frame_stride[p];
        }
        a.w = E->w; a.h = E->h; a.bytes = E->fi.depth > 8 ? 2 : 1; a.bits = E->fi.depth;
        a.hsub = E->fi.hsub; a.vsub = E->fi.vsub; a.nh = E->nh; a.nv = E->nv; a.nslices = ns;
        a.cap = E->cap; a.states = E->states; a.sizes = E->sizes; a.crcs = E->crcs;
        a.tables = E->tables;
        a.tok = E->tok; a.tok_len = E->tok_len; a.raw = E->raw; a.raw_cap = rcap; a.nraw = E->nraw;
        for (int k = 0; k < 5; ++k) a.qthr[k] = k < E->quant.n ? E->quant.thr[k] : 1024;
        a.qL = E->quant.levels();
        a.nctx = E->quant.contexts();
        a.state_bytes = E->state_bytes();
        const int nwg = (ns + 63) / 64;
        PP_HIP(hipMemsetAsync(E->states, 128, (size_t)E->state_bytes() * nwg * 64, st));  // every context of every slice: 128
        if (a.bytes == 2)
            hipLaunchKernelGGL(ffv1_model_kernel<uint16_t>, dim3((unsigned)E->rows_max, nwg), dim3(256), 0, st, a);
        else
            hipLaunchKernelGGL(ffv1_model_kernel<uint8_t>, dim3((unsigned)E->rows_max, nwg), dim3(256), 0, st, a);
        a.lpw = ffv1_lanes_per_wave(64);
        if (const char *e = PP_KNOB("PIXPATH_FFV1_DEBUG")) a.debug = std::atoi(e);
        hipLaunchKernelGGL(ffv1_code_kernel, dim3((ns + a.lpw - 1) / a.lpw), dim3(64), 0, st, a);
        // the byte machine is one dependent chain per slice over its records; full
        // waves measured best (64 / 16 / 8 lanes: 16.3 / 18.1 / 25.2 ms per 600 frames)
        a.rlpw = 64;
        if (const char *e = PP_KNOB("PIXPATH_FFV1_RLPW")) a.rlpw = std::max(1, std::min(64, std::atoi(e)));
        hipLaunchKernelGGL(ffv1_resolve_kernel, dim3((ns + a.rlpw - 1) / a.rlpw), dim3(64), 0, st, a);
        PP_HIP(hipGetLastError());
        ++E->launches;
        sizes.resize(ns);
        off.resize(ns);
        PP_HIP(hipMemcpyAsync(sizes.data(), E->sizes, sizeof(int64_t) * ns, hipMemcpyDeviceToHost, st));
        PP_HIP(hipStreamSynchronize(st));
        bool short_of_records = false;
        for (int i = 0; i < ns && !short_of_records; ++i) short_of_records = sizes[i] < 0;
        if (short_of_records && rcap < E->full_raw && m > 1) {
            m = (m + 1) / 2;  // the same frames again, twice the records per slice
            continue;
        }
        int64_t part = 0;
        for (int f = 0; f < m; ++f) {
            int64_t fsz = 0;
            for (int s = 0; s < per; ++s) {
                const int64_t n = sizes[f * per + s];
                if (n < 0)
                    PP_FAIL(PP_ERR_NOMEM, "frame %d slice %d exceeds its %lld-byte buffer", f0 + f, s,
                            (long long)(rcap * 4));
                if (n + 8 >= ((int64_t)1 << 24))  // the footer's 24-bit size field (ffv1enc.c asserts the same)
                    PP_FAIL(PP_ERR_UNSUPPORTED, "frame %d slice %d: %lld bytes exceed the 24-bit slice size", f0 + f,
                            s, (long long)n);
                off[f * per + s] = total + part + fsz;
                fsz += n + 8;
            }
            frame_sizes[f0 + f] = fsz;
            part += fsz;
        }
        if (int rc = pk_reserve(E, total + part, total, st)) return rc;
        PP_HIP(hipMemcpyAsync(E->off, off.data(), sizeof(int64_t) * ns, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(ffv1_pack_kernel, dim3(ns), dim3(256), 0, st, reinterpret_cast<const uint8_t *>(E->raw),
                           rcap * 4, E->sizes, E->crcs, E->off, E->pk,
                           reinterpret_cast<const uint32_t *>(E->tables + 512));
        PP_HIP(hipGetLastError());
        // the next launch reuses the records, the sizes and the offsets
        PP_HIP(hipStreamSynchronize(st));
        total += part;
        f0 += m;
    }
    E->pk_len = total;
    if (packets) *packets = E->pk;
    return total;
}

extern "C" int pp_ffv1_encoder_reserve(pp_ffv1_enc *E, int64_t packet_bytes) {
    if (!E || packet_bytes < 0) PP_FAIL(PP_ERR_INVALID, "bad argument");
    if (!E->ctx) PP_FAIL(PP_ERR_INVALID, "host-only encoder");
    PP_HIP(hipSetDevice(E->ctx->device));
    return pk_reserve(E, packet_bytes, 0, nullptr);
}

extern "C" int pp_ffv1_encode_stats(const pp_ffv1_enc *E, int *launches) {
    if (!E || !launches) PP_FAIL(PP_ERR_INVALID, "null argument");
    *launches = E->launches;
    return PP_OK;
}

extern "C" int64_t pp_ffv1_encode(pp_ffv1_enc *E, const pp_frames *src, int nframes, uint8_t *dst, int64_t dst_cap,
                                  int64_t *frame_sizes, void *stream) {
    if (!E || !src || !dst || !frame_sizes || nframes < 0) PP_FAIL(PP_ERR_INVALID, "null argument");
    const uint8_t *pk = nullptr;
    const int64_t total = pp_ffv1_encode_packets(E, src, nframes, frame_sizes, &pk, stream);
    if (total <= 0) return total;
    if (total > dst_cap) PP_FAIL(PP_ERR_NOMEM, "packets need %lld bytes, dst holds %lld", (long long)total, (long long)dst_cap);
    hipStream_t st = static_cast<hipStream_t>(stream);
    PP_HIP(hipMemcpyAsync(dst, pk, total, hipMemcpyDeviceToDevice, st));
    PP_HIP(hipStreamSynchronize(st));
    return total;
}
