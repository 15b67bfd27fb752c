// strip_kernel: the common-case scaler (every plane in 256-column strips,
// 16-B aligned source rows, <= 8 vertical tap pairs, <= 10-bit samples).
// Included by strip_u16.hip / strip_u8.hip, which instantiate it per source
// sample type; the launch code is in scale.hip.
//
// Same strip/segment/chunk walk and LDS layout as scale_kernel, but every
// loop is wave-uniform (wave = row group, lane = 4 adjacent columns), so the
// control flow is scalar branches instead of exec-mask bookkeeping:
//   H pass: one lane computes 4 adjacent output columns of a row PAIR.  The 4
//     windows share one 8-B aligned base in the staged row (hbase4), read as
//     HW dwords with ds_read_b64 (one read serves all 4 outputs); per output
//     the taps are re-laid over those dwords (hcoefw, zero outside its
//     window), so each output is HW v_dot2_i32_i16 with no realignment, and
//     the 8 results go to the window as one ds_write_b128.
//   V pass: a wave owns an output row; the row records (window base row + tap
//     pairs, a padded [dh][16] table) of several rows come through the scalar
//     cache at once (SGPR operands of v_dot2, one exposed scalar-load latency
//     per group of rows), the window rows through ds_read_b128 (4 columns x 2
//     rows), one 8-B store per row.
//   Staging: the next chunk's new source rows are loaded into registers right
//     after the chunk-start barrier and written to LDS right after the window
//     barrier (when the H pass has released the staging rows).  The wave
//     issues no other vector-memory op in between, so the wait for those
//     loads never covers its own V-pass stores (vmcnt counts loads and stores
//     in issue order).
// Measured (profiles/r2): the per-row dependent scalar load of the V-pass row
// record and the register budget (104 VGPRs = 4 workgroups/CU) were what kept
// the round-1 kernel at 0.50 of the HBM roofline.
#pragma once
#include "scale_dev.hpp"

namespace pp {

// 16-B staging chunks per lane prefetched into registers: 3 covers the new
// source rows of an upscale chunk; 16-bit sources with wide H windows (HW >= 8:
// downscales, ~2 new source rows per output row) get PIXPATH_STRIP_PF_WIDE so
// the staging of a chunk is not mostly synchronous loads in commit()
// (config 3, 2160p yuv422p10le -> 1080p: 5.94 -> 4.82 ms; 8-bit sources stage
// 16 samples per chunk and lose slightly with 6: 3.32 -> 3.40 ms)
#ifndef PIXPATH_STRIP_PF_WIDE
#define PIXPATH_STRIP_PF_WIDE 6
#endif
#ifndef PIXPATH_STRIP_PF_U8_WIDE
#define PIXPATH_STRIP_PF_U8_WIDE 3
#endif
#ifndef PIXPATH_STRIP_PF_NARROW
#define PIXPATH_STRIP_PF_NARROW 3
#endif
template <int HW, int SB>
constexpr int strip_pf() {
    return HW >= 8 ? (SB == 2 ? PIXPATH_STRIP_PF_WIDE : PIXPATH_STRIP_PF_U8_WIDE) : PIXPATH_STRIP_PF_NARROW;
}
template <int PF>
struct StripPrefetch {
    uint4 v[PF];
};

// Waves per SIMD the register allocation is bounded for: 6 (80 VGPRs, the LDS
// limit of the config-2 plan: 6 workgroups/CU) where that needs no spill,
// else 4 (128 VGPRs) or 3 (168 VGPRs, the widest H windows).  tools/check_spills.sh checks every instance.
template <int SB, int OUTB, int HW, int VTM>
constexpr int strip_min_waves() {
    return HW >= 10 ? 3 : (VTM <= 5 && HW <= (OUTB == 10 && SB == 2 ? 6 : 4)) ? 6 : 4;
}

// 4 adjacent outputs of a row at column xo (8-bit bytes or 16-bit samples)
template <int BITS>
__device__ inline void store4(uint8_t *drow, int xo, const int o[4], bool vec, int dw) {
    if constexpr (BITS == 8) {
        if (vec) {
            // opaque bytes: two clamped 8-bit results otherwise fold into
            // v_ashr_pk_u8_i32, which leaves its destination's high half as it
            // was, and the OR then keeps those stale bits in bytes 2 and 3
            // (tests/test_gpu_chain.py caught it; cpvs.hip has the same guard)
            uint32_t b[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                b[j] = (uint32_t)o[j];
                asm volatile("" : "+v"(b[j]));
            }
            *reinterpret_cast<uint32_t *>(drow + xo) = b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (xo + j < dw) drow[xo + j] = (uint8_t)o[j];
        }
    } else {
        uint16_t *d16 = reinterpret_cast<uint16_t *>(drow);
        if (vec) {
            uint2 v;
            v.x = (uint32_t)o[0] | ((uint32_t)o[1] << 16);
            v.y = (uint32_t)o[2] | ((uint32_t)o[3] << 16);
            *reinterpret_cast<uint2 *>(d16 + xo) = v;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (xo + j < dw) d16[xo + j] = (uint16_t)o[j];
        }
    }
}

// clamp(acc >> SH, 0, MX) of two 32-bit V-pass sums, packed as two 16-bit
// samples (a low, b high): the high halves of both sums in one v_perm, then
// v_pk_ashrrev_i16 / v_pk_max_i16 / v_pk_min_i16 -- 4 VALU per pair instead
// of 2 shifts, 2 v_med3 and a v_lshl_or.  Exact: acc >> 16 is the sum's exact
// signed high half, and (acc >> 16) >> (SH - 16) == acc >> SH.
// (not in the product: it pushes the config-2 instance to 2 spilled VGPRs)
#ifndef PIXPATH_PACKED_CLAMP
#define PIXPATH_PACKED_CLAMP 0
#endif
template <int SH, int MX>
__device__ inline uint32_t clamp_pack16(int a, int b) {
    static_assert(SH >= 16 && SH < 32 && MX < 32768, "packed clamp range");
    v2i16 x = __builtin_bit_cast(v2i16, __builtin_amdgcn_perm((uint32_t)b, (uint32_t)a, 0x07060302u));
    if constexpr (SH > 16) x = x >> (v2i16){(short)(SH - 16), (short)(SH - 16)};
    x = __builtin_elementwise_max(x, (v2i16){0, 0});
    x = __builtin_elementwise_min(x, (v2i16){(short)MX, (short)MX});
    return __builtin_bit_cast(uint32_t, x);
}

// FUSE == 1 (GENERIC_UYVY plans: scale straight into uyvy422, swscale's
// yuv2packedX with its flat 1 << 18 rounding): every plane stores its 8-bit
// samples into the one packed row, byte J.pk_off + x * J.pk_step (Y: 1, 2;
// U: 0, 4; V: 2, 4) -- no planar scratch, no interleave pass.
// FUSE >= 8 (chain plans, pp_scale_chain_plan_create; register budget
// strip_chain_min_waves): 0 = plain plan; 8 / 10 = the
// two-stage chain of create_avpvs_segment -- this kernel's 8-bit (OUTB == 8)
// output is the overlay's yuv420p, and the per-plane mode J.fuse applies
// libavfilter's auto-inserted yuv420p -> target conversion (FUSE-bit output)
// before anything reaches HBM:
//   fuse 0: stored as is (8-bit target, identity second stage);
//   fuse 1: identity second stage into FUSE bits (x << 7 -> yuv2planeX);
//   fuse 2: chroma 4:2:0 -> 4:2:2: the 8-bit rows go to an LDS ring (ring2,
//     15-bit intermediates = hScale8To15 of the identity H filter), and after
//     each chunk the second stage's vertical filter (vrow2, chunk2 tables)
//     emits every output row whose taps are all in the ring.
// TW = strip width = threads: 256 (4 waves, one per row group) or 512 (8 waves:
// row group wave >> 1, column half wave & 1; same 4 outputs per lane, half the
// strips, so half the column-halo staging and 1-KB contiguous row stores)
// Chain plans (FUSE >= 8): the same per-instance budget rule, with the ring2
// path's extra registers -- 6 waves where that is spill-free (config 4's
// <u16, 8, 4, 3, 10>: 79 VGPRs), 4 for windows up to 10 dwords, else 3
// (tools/check_spills.sh).  Was 3 for every chain instance: 3 workgroups per
// CU although the plan's LDS (~25 KB) allows 6.
template <int HW, int VTM>
constexpr int strip_chain_min_waves() {
    return (HW <= 4 && VTM <= 3) ? 6 : ((HW <= 10 && VTM <= 5) || (HW == 12 && VTM <= 3)) ? 4 : 3;
}
#ifndef PIXPATH_LUMA9_WAVES
#define PIXPATH_LUMA9_WAVES 6
#endif
#ifndef PIXPATH_CHROMA11_WAVES
#define PIXPATH_CHROMA11_WAVES 7
#endif
// FUSE 9 / 11 (a chain's luma / chroma launch alone): their own budgets where
// the window is narrow
template <int HW, int VTM, int FUSE>
constexpr int strip_fused_min_waves() {
    return FUSE == 9 && HW <= 4 && VTM <= 3    ? PIXPATH_LUMA9_WAVES
           : FUSE == 11 && HW <= 4 && VTM <= 3 ? PIXPATH_CHROMA11_WAVES
                                               : strip_chain_min_waves<HW, VTM>();
}
// Instances with register room for the clamped V-pass copy (a second
// instantiation of the row loop): the rest keep the per-lane path rather than
// spill (tools/check_spills.sh: 8-bit sources into 8-bit rows with 4-dword
// windows, chain plans with 10+ dword windows spilled 1-5 VGPRs with it).
template <typename ST, int OUTB, int HW, int VTM, int FUSE>
constexpr bool strip_clamp_path() {
    return !(FUSE >= 8 && HW >= 10) && !(sizeof(ST) == 1 && OUTB == 8 && HW == 4 && (FUSE >= 8 || VTM >= 5));
}

template <typename ST, int OUTB, int HW, int VTM, int FUSE = 0, int TW = 256>
__global__ __launch_bounds__(TW, (FUSE >= 8 ? strip_fused_min_waves<HW, VTM, FUSE>() : strip_min_waves<(int)sizeof(ST), OUTB, HW, VTM>())) void strip_kernel(const ScaleArgs a) {
    static_assert(TW == 256 || TW == 512, "strip width");
    // DIRECT (8-dword windows: the 2:1 downscales of config 3): no staged
    // source rows -- a lane loads its window's 16 source samples of a row
    // straight into registers for the H pass (one 16-B load of 8-bit samples,
    // two of 16-bit ones), so the plan's LDS is the V window ring alone (the
    // staged rows were two thirds of it and kept the chunks at 8 rows).
    // 8-bit sources only: config 3's 10-bit source measured slower direct
    // (4.85 vs 4.73 ms at 24-row chunks, profiles/r5/config3_direct.txt)
    constexpr bool DIRECT = sizeof(ST) == 1 && HW == 8 && FUSE == 0;
    extern __shared__ __align__(16) uint16_t lds[];
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int frame = L / a.tiles;
    int t = L - frame * a.tiles;
    int p = 0;
    if (a.nplanes > 1 && t >= a.pl[1].tile_base) p = 1;
    if (a.nplanes > 2 && t >= a.pl[2].tile_base) p = 2;
    const PlaneJob &J = a.pl[p];
    t -= J.tile_base;
    const int seg = t / J.tiles_x, tx = t - seg * J.tiles_x;
    const int x0 = tx * TW, nx = min(TW, J.dw - x0);
    const int c0 = as_kconst<int32_t>(J.tile_c0)[tx], cn = as_kconst<int32_t>(J.tile_cn)[tx];
    // chunk tables through the scalar cache: no vector-memory wait at chunk starts
    const kconst int32_t *chunk_lo = as_kconst<int32_t>(J.chunk_lo), *chunk_hi = as_kconst<int32_t>(J.chunk_hi);
    const int S = J.S;
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // row group (H-pass row pairs and V-pass rows strided by 4); at TW = 512
    // waves 2r and 2r+1 are row group r, left and right 256 columns
    const int rg = TW == 512 ? wave >> 1 : wave;
    const int cx = (tid & (TW / 4 - 1)) * 4;
    uint16_t *src_t = lds;                                                  // [maxnew][S]
    uint32_t *win = reinterpret_cast<uint32_t *>(lds + J.maxnew * S);       // [ring/2][TW] row pairs
    // FUSE, fuse 2: the second stage's input rows as bytes, a circular ring of
    // J.r2mask + 1 rows ([row & r2mask][TW] bytes): a lane stores its 4 bytes
    // of a row in one conflict-free dword, and no row is ever moved
    uint8_t *ring2b = reinterpret_cast<uint8_t *>(win + (J.ring >> 1) * TW);
    const kconst int32_t *chunk2 = as_kconst<int32_t>(J.chunk2);            // [nch][4]: lo2, hi2, base2, keep2
    const ST *sbase = reinterpret_cast<const ST *>(a.src[p] + frame * a.sfs[p]);
    uint8_t *dbase = a.dst[p] + frame * a.dfs[p];

    // ---- horizontal taps of this lane's 4 columns over its HW-dword window ----
    constexpr int hshift = sizeof(ST) == 1 ? 7 : 9;
    const int g = tx * (TW / 4) + (tid & (TW / 4 - 1));
    const int hb = J.hbase4[g];
    v2i16 hc[4][HW];
    {
        const int4 *hp4 = reinterpret_cast<const int4 *>(J.hcoefw + (int64_t)g * 4 * HW);
#pragma unroll
        for (int i = 0; i < HW; ++i) {
            const int4 v = hp4[i];
            const int e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) hc[(4 * i + q) / HW][(4 * i + q) % HW] = __builtin_bit_cast(v2i16, e[q]);
        }
        // consume the taps here, so their vmcnt wait is placed before the chunk
        // loop (inside it, the wait would also cover the previous chunk's stores)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int d = 0; d < HW; ++d) asm volatile("" ::"v"(hc[j][d]));
        asm volatile("" ::"v"(hb));
    }

    // ---- staging (16-B loads through the plane's buffer resource) ----------
    // (DIRECT: the plan passes maxnew = 0, so `win` starts the LDS)
    constexpr int CH = 16 / sizeof(ST);
    const int cpr = (cn + CH - 1) / CH;  // 16-B chunks per staged row (<= TW, host-checked)
    const int64_t sls = a.sls[p];
    const int sw = J.sw;
    const int64_t last_row = std::min<int64_t>(sls, ((int64_t)sw * sizeof(ST) + 15) & ~int64_t(15));
    const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(sbase, (int)((int64_t)(J.sh - 1) * sls + last_row));
    const int cbyte = c0 * (int)sizeof(ST);
    const int s_rstep = TW / cpr;
    const int s_r0 = tid / cpr, s_ch = tid - s_r0 * cpr;
    const bool s_on = s_r0 < s_rstep;
    const int s_lds = s_r0 * S + s_ch * CH;
    const int s_goff = s_r0 * (int)sls + cbyte + s_ch * 16;
    constexpr int kStripPF = strip_pf<HW, (int)sizeof(ST)>();
    auto prefetch = [&](StripPrefetch<kStripPF> &pf, int from, int hi_) {
        const int nrow = hi_ - from;
#pragma unroll
        for (int k = 0; k < kStripPF; ++k) {
            const int r = s_r0 + k * s_rstep;
            pf.v[k] = bload16(rs, (s_on && r < nrow) ? s_goff + (from + k * s_rstep) * (int)sls : kOobOff);
        }
    };
    auto commit = [&](const StripPrefetch<kStripPF> &pf, int from, int hi_) {
        const int nrow = hi_ - from;
        if (!s_on) return;
#pragma unroll
        for (int k = 0; k < kStripPF; ++k)
            if (s_r0 + k * s_rstep < nrow) store_raw16<ST>(src_t + s_lds + k * s_rstep * S, pf.v[k]);
        for (int k = kStripPF; s_r0 + k * s_rstep < nrow; ++k)
            store_raw16<ST>(src_t + s_lds + k * s_rstep * S, bload16(rs, s_goff + (from + k * s_rstep) * (int)sls));
    };

    // 4 outputs of one staged row (15-bit intermediates, hScale*To15 clip)
    auto hrow4 = [&](const uint16_t *row, int out[4]) {
        const uint16_t *sp = row + hb;
        uint32_t w[HW];
#pragma unroll
        for (int d = 0; d + 1 < HW; d += 2) {
            const uint2 v = *reinterpret_cast<const uint2 *>(sp + 2 * d);
            w[d] = v.x;
            w[d + 1] = v.y;
        }
        if constexpr (HW & 1) w[HW - 1] = *reinterpret_cast<const uint32_t *>(sp + 2 * (HW - 1));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            int acc = dot2_first(__builtin_bit_cast(v2i16, w[0]), hc[j][0]);
#pragma unroll
            for (int d = 1; d < HW; ++d) acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16, w[d]), hc[j][d], acc, false);
            acc >>= hshift;
            out[j] = acc < 32767 ? acc : 32767;
        }
    };

    // the same without the clamp: a row pair's results are packed by
    // v_cvt_pk_i16_i32, whose saturation is the clamp (the host admits a plan
    // to this kernel only if no output can fall below -32768, strip_h_sat_ok)
    auto hrow4_raw = [&](const uint16_t *row, int out[4]) {
        const uint16_t *sp = row + hb;
        uint32_t w[HW];
#pragma unroll
        for (int d = 0; d + 1 < HW; d += 2) {
            const uint2 v = *reinterpret_cast<const uint2 *>(sp + 2 * d);
            w[d] = v.x;
            w[d + 1] = v.y;
        }
        if constexpr (HW & 1) w[HW - 1] = *reinterpret_cast<const uint32_t *>(sp + 2 * (HW - 1));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            int acc = dot2_first(__builtin_bit_cast(v2i16, w[0]), hc[j][0]);
#pragma unroll
            for (int d = 1; d < HW; ++d) acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16, w[d]), hc[j][d], acc, false);
            out[j] = acc >> hshift;
        }
    };
    // rows a (low halves) and b (high halves) of 4 columns, each clamped to 32767
    auto pack_pair = [](const int oa[4], const int ob[4]) {
        uint4 v;
        v.x = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_i16(oa[0], ob[0]));
        v.y = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_i16(oa[1], ob[1]));
        v.z = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_i16(oa[2], ob[2]));
        v.w = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_i16(oa[3], ob[3]));
        return v;
    };

    int y_begin = seg * J.seg_h, y_end = min(J.dh, y_begin + J.seg_h);
    int r2lo = 0, r2hi = 0;  // fuse 2: the second-stage rows this segment stores
    if constexpr (FUSE >= 8 && FUSE != 9) {
        if (J.fuse == 2) {  // first-stage rows of the segment plus the halo its second-stage rows read
            const kconst int32_t *sg = as_kconst<int32_t>(J.seg2) + 4 * seg;
            y_begin = sg[0];
            y_end = sg[1];
            r2lo = sg[2];
            r2hi = sg[3];
        }
    }
    const int cho = J.cho;
    int next_src = chunk_lo[y_begin / cho];
    int base = next_src & ~1;
    StripPrefetch<kStripPF> pf;
    // the first chunk's rows are staged before the loop; every later chunk's
    // rows are loaded right after the chunk-start barrier of the chunk before
    // and written to LDS right after its window barrier (src_t is free then).
    // Between those two points the wave issues no vector-memory op, so the
    // wait for the loads never covers this wave's V-pass stores (vmcnt is
    // in-order over loads and stores).
    if constexpr (!DIRECT) {
        prefetch(pf, next_src, chunk_hi[y_begin / cho]);
        commit(pf, next_src, chunk_hi[y_begin / cho]);
    }
    const bool lane_any = cx < nx, lane_full = cx + 4 <= nx;
    const int xo = x0 + cx;
    // clamped V pass (wave-uniform): when the strip ends on a 4-column group
    // and rows take vector stores, a lane past the strip's last group reads
    // that group's window columns and stores its outputs again -- the same
    // bytes to the same address -- so the V-pass row loop has no per-lane
    // branch (a divergent `continue` per stored row turned every unrolled row
    // group into exec-mask bookkeeping: more SALU than VALU instructions in
    // the chain kernel, profiles/r3/chain_ablation.txt)
    const bool clamp = (nx & 3) == 0 && a.vec_dst;
    const int cxv = clamp ? min(cx, nx - 4) : cx;
    const int xov = x0 + cxv;
    const int64_t dls = a.dls[p];
    const int vtp = J.vtp;
    const int jdw = J.dw;
    // FUSE 9 / 11: a 10-bit chain plan's luma launch alone (fuse 1: no ring2,
    // no second stage) / chroma launch alone (fuse 2), the mode a compile-time
    // constant
    const int jfuse = FUSE == 9 ? 1 : FUSE == 11 ? 2 : FUSE >= 8 ? J.fuse : 0;
    constexpr int OUT2 = FUSE == 9 || FUSE == 11 ? 10 : FUSE;  // the chain's output bits
    const kconst int32_t *vrow = as_kconst<int32_t>(J.vrow16);
    // the V pass's rounding constant in a VGPR: the first v_dot2 of an output
    // takes it as its accumulator operand (dot2_sv; a literal accumulator cost
    // a v_mov per output and row)
    int kround = 1 << (10 + 16 - OUTB);
    asm volatile("" : "+v"(kround));
    for (int y0 = y_begin; y0 < y_end; y0 += cho) {
        const int ci = y0 / cho;
        const int lo = chunk_lo[ci], hi = chunk_hi[ci];
        if (next_src < lo) next_src = lo;
        const int nnew = hi - next_src;
        const int nbase = lo & ~1;
        const int keep = next_src > nbase ? (next_src - nbase + 1) >> 1 : 0;
        const int shift = (nbase - base) >> 1;
        if (!(PP_ABLATE(a.debug) & 8)) __syncthreads();  // staged rows visible; every wave has left the previous V pass
        const int after = nnew > 0 ? hi : next_src;
        const bool more = y0 + cho < y_end;
        const int nfrom = more ? max(after, chunk_lo[ci + 1]) : 0, nhi = more ? chunk_hi[ci + 1] : 0;
        if (!DIRECT && more && !(PP_ABLATE(a.debug) & 2)) prefetch(pf, nfrom, nhi);
        // kept row pairs move down to the window start, each column by its own
        // lane in increasing order (no lane reads a slot already overwritten)
        bool moved = false;
        if (shift > 0) {
            for (int k = 0; k < keep; ++k) win[k * TW + tid] = win[(k + shift) * TW + tid];
            moved = true;
        }
        if (moved) __syncthreads();
        base = nbase;
        // ---- horizontal pass: row pairs of the window, wave-strided ----------
        if (nnew > 0 && (PP_ABLATE(a.debug) & 4)) next_src = hi;
        if (DIRECT && nnew > 0 && !(PP_ABLATE(a.debug) & 4)) {
            // window row i = source row base + i; a lane's 16 samples at its
            // window base (dword aligned: c0 % 16 == 0, hb % 4 == 0)
            const int i0 = next_src - base;
            const int kf0 = (i0 + 1) >> 1, kf1 = (i0 + nnew) >> 1;
            const int hoff = cbyte + hb * (int)sizeof(ST);
            struct Win {
                uint4 v[sizeof(ST)];
            };
            auto ld = [&](int i) {
                Win r;
                const int off = (base + i) * (int)sls + hoff;
#pragma unroll
                for (int k = 0; k < (int)sizeof(ST); ++k) r.v[k] = bload16(rs, off + 16 * k);
                return r;
            };
            auto hregs = [&](const Win &r, int out[4]) {  // hrow4 on register-held samples
                uint32_t w[HW];
                if constexpr (sizeof(ST) == 1) {
                    const uint32_t d4[4] = {r.v[0].x, r.v[0].y, r.v[0].z, r.v[0].w};
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        w[2 * m] = __builtin_amdgcn_perm(0u, d4[m], 0x0c010c00u);
                        w[2 * m + 1] = __builtin_amdgcn_perm(0u, d4[m], 0x0c030c02u);
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        w[4 * k] = r.v[k].x; w[4 * k + 1] = r.v[k].y; w[4 * k + 2] = r.v[k].z; w[4 * k + 3] = r.v[k].w;
                    }
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    int acc = dot2_first(__builtin_bit_cast(v2i16, w[0]), hc[j][0]);
#pragma unroll
                    for (int d = 1; d < HW; ++d)
                        acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16, w[d]), hc[j][d], acc, false);
                    out[j] = acc >> hshift;  // clamped by the caller (pack_pair or min)
                }
            };
            auto pair_out = [&](int k, const Win &ra, const Win &rb) {
                int oa[4], ob[4];
                hregs(ra, oa);
                hregs(rb, ob);
                *reinterpret_cast<uint4 *>(win + k * TW + cx) = pack_pair(oa, ob);
            };
            if ((i0 & 1) && rg == ((i0 >> 1) & 3)) {  // high row of a kept pair
                int o[4];
                hregs(ld(i0), o);
                uint16_t *w16 = reinterpret_cast<uint16_t *>(win + (i0 >> 1) * TW + cx);
#pragma unroll
                for (int j = 0; j < 4; ++j) w16[2 * j + 1] = static_cast<uint16_t>(min(o[j], 32767));
            }
            if (((i0 + nnew) & 1) && rg == (kf1 & 3)) {  // low row of the last pair
                int o[4];
                hregs(ld(i0 + nnew - 1), o);
                uint4 v;
                v.x = min(o[0], 32767) & 0xffff; v.y = min(o[1], 32767) & 0xffff;
                v.z = min(o[2], 32767) & 0xffff; v.w = min(o[3], 32767) & 0xffff;
                *reinterpret_cast<uint4 *>(win + kf1 * TW + cx) = v;
            }
            int k = kf0 + rg;
            for (; k + 4 < kf1; k += 8) {  // two pairs a step: four row loads in flight
                const Win a0 = ld(2 * k), a1 = ld(2 * k + 1), b0 = ld(2 * k + 8), b1 = ld(2 * k + 9);
                pair_out(k, a0, a1);
                pair_out(k + 4, b0, b1);
            }
            if (k < kf1) pair_out(k, ld(2 * k), ld(2 * k + 1));
            next_src = hi;
        }
        if (!DIRECT && nnew > 0 && !(PP_ABLATE(a.debug) & 4)) {
            const int i0 = next_src - base;
            const int kf0 = (i0 + 1) >> 1, kf1 = (i0 + nnew) >> 1;
            if ((i0 & 1) && rg == ((i0 >> 1) & 3)) {  // high row of a kept pair
                int o[4];
                hrow4(src_t, o);
                uint16_t *w16 = reinterpret_cast<uint16_t *>(win + (i0 >> 1) * TW + cx);
#pragma unroll
                for (int j = 0; j < 4; ++j) w16[2 * j + 1] = static_cast<uint16_t>(o[j]);
            }
            if (((i0 + nnew) & 1) && rg == (kf1 & 3)) {  // low row of the last pair
                int o[4];
                hrow4(src_t + (nnew - 1) * S, o);
                uint4 v;
                v.x = o[0] & 0xffff; v.y = o[1] & 0xffff; v.z = o[2] & 0xffff; v.w = o[3] & 0xffff;
                *reinterpret_cast<uint4 *>(win + kf1 * TW + cx) = v;
            }
            for (int k = kf0 + rg; k < kf1; k += 4) {
                const int ra = 2 * k - i0;
                int oa[4], ob[4];
                hrow4_raw(src_t + ra * S, oa);
                hrow4_raw(src_t + (ra + 1) * S, ob);
                *reinterpret_cast<uint4 *>(win + k * TW + cx) = pack_pair(oa, ob);
            }
            next_src = hi;
        }
        if (!(PP_ABLATE(a.debug) & 8)) __syncthreads();  // window complete; src_t is free
        if (!DIRECT && more && nhi > nfrom && !(PP_ABLATE(a.debug) & 2)) commit(pf, nfrom, nhi);
        // ---- vertical pass: one output row per wave --------------------------
        // raised priority while the wave issues its output rows: the other
        // waves' H pass never starves the write stream (-2 %, profiles/r2)
        __builtin_amdgcn_s_setprio(1);
        const int ny = min(cho, y_end - y0);
        // VT (= vtp) tap pairs, compile-time per instance: every window read of
        // a row is in flight before the first v_dot2 waits on one
        auto vpass = [&](auto vt_c, auto cl_c) {
            constexpr int VT = decltype(vt_c)::value;
            constexpr bool CL = decltype(cl_c)::value;  // clamped lanes: no per-lane branch
            const int vx = CL ? cxv : cx, vxo = CL ? xov : xo;
            // row records (window base row + VT tap pairs) of G rows at a time
            // through the scalar cache: one exposed scalar-load latency per
            // group, not per row (the ds_reads of a row depend on its base)
            constexpr int G = VT <= 2 ? 8 : VT <= 5 ? 4 : 2;
            // 8-bit rows: the ordered dither's accumulator inits, once per
            // chunk.  A wave's rows are y0 + rg + 4k, so y & 7 takes two values
            // -- row g0 + 4i of a group is phase i & 1 (G is even) -- and the
            // lane's 4 columns are fixed: the two phases' inits are computed
            // here instead of a scalar dither load, a 64-bit rotate and 4
            // byte extracts per row (11 of the 35 VALU of a FUSE-9 row)
            // (config 4's 10-bit-source instances only: the 8-VGPR table spills
            // the other 8-bit-output instances at their register budgets)
            constexpr bool DACPRE = OUTB == 8 && sizeof(ST) == 2 && (FUSE == 9 || FUSE == 11);
            int dac[2][4];
            if constexpr (DACPRE) {
#pragma unroll
                for (int ph = 0; ph < 2; ++ph) {
                    uint32_t d4 = 0x40404040u;  // flat 64 without dither
                    if (a.dither) {
                        const uint64_t rv = as_kconst<uint64_t>(c_dither64)[(y0 + rg + 4 * ph) & 7];
                        const int rot = ((vxo + J.dither_off) & 7) * 8;
                        d4 = (uint32_t)(rot ? (rv >> rot) | (rv << (64 - rot)) : rv);
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) dac[ph][j] = (int)((d4 >> (8 * j)) & 0xffu) << 12;
                }
            }
            for (int g0 = rg; g0 < ny; g0 += 4 * G) {
                int vb[G];
                int32_t cf[G][VT];
#pragma unroll
                for (int i = 0; i < G; ++i) {
                    const int rr = min(g0 + 4 * i, ny - 1);  // clamped: loads stay inside the table
                    const kconst int32_t *row = vrow + (int64_t)(y0 + rr) * 16;
                    vb[i] = row[0];
#pragma unroll
                    for (int j = 0; j < VT; ++j) cf[i][j] = row[1 + j];
                }
#pragma unroll
                for (int i = 0; i < G; ++i) {
                    const int yy = g0 + 4 * i;
                    if (yy >= ny) break;
                    const int y = y0 + yy;
                    uint8_t *drow_p = dbase + (int64_t)y * dls;
                    const uint4 *rp = reinterpret_cast<const uint4 *>(win + ((vb[i] - nbase) >> 1) * TW + vx);
                    uint4 q[VT];
#pragma unroll
                    for (int j = 0; j < VT; ++j) q[j] = rp[j * (TW / 4)];
                    int acc[4];
                    // the first tap pair onto the rounding constant (16-bit rows)
                    // or the row's dither init (8-bit rows), both VGPRs
                    if constexpr (OUTB == 8 && !DACPRE) {
                        // ordered dither: the row's 8 bytes (scalar load, y is wave-uniform)
                        // rotated to the lane's first column; flat 64 without dither
                        uint32_t d4 = 0x40404040u;
                        if (a.dither) {
                            const uint64_t rv = as_kconst<uint64_t>(c_dither64)[y & 7];
                            const int rot = ((vxo + J.dither_off) & 7) * 8;
                            d4 = (uint32_t)(rot ? (rv >> rot) | (rv << (64 - rot)) : rv);
                        }
                        int dj[4];
#pragma unroll
                        for (int j = 0; j < 4; ++j) dj[j] = (int)((d4 >> (8 * j)) & 0xffu) << 12;
                        acc[0] = dot2_sv(__builtin_bit_cast(v2i16, q[0].x), cf[i][0], dj[0]);
                        acc[1] = dot2_sv(__builtin_bit_cast(v2i16, q[0].y), cf[i][0], dj[1]);
                        acc[2] = dot2_sv(__builtin_bit_cast(v2i16, q[0].z), cf[i][0], dj[2]);
                        acc[3] = dot2_sv(__builtin_bit_cast(v2i16, q[0].w), cf[i][0], dj[3]);
                    } else if constexpr (OUTB == 8) {
                        acc[0] = dot2_sv(__builtin_bit_cast(v2i16, q[0].x), cf[i][0], dac[i & 1][0]);
                        acc[1] = dot2_sv(__builtin_bit_cast(v2i16, q[0].y), cf[i][0], dac[i & 1][1]);
                        acc[2] = dot2_sv(__builtin_bit_cast(v2i16, q[0].z), cf[i][0], dac[i & 1][2]);
                        acc[3] = dot2_sv(__builtin_bit_cast(v2i16, q[0].w), cf[i][0], dac[i & 1][3]);
                    } else {
                        acc[0] = dot2_sv(__builtin_bit_cast(v2i16, q[0].x), cf[i][0], kround);
                        acc[1] = dot2_sv(__builtin_bit_cast(v2i16, q[0].y), cf[i][0], kround);
                        acc[2] = dot2_sv(__builtin_bit_cast(v2i16, q[0].z), cf[i][0], kround);
                        acc[3] = dot2_sv(__builtin_bit_cast(v2i16, q[0].w), cf[i][0], kround);
                    }
#pragma unroll
                    for (int j = 1; j < VT; ++j) {
                        const v2i16 c2 = __builtin_bit_cast(v2i16, cf[i][j]);
                        acc[0] = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16, q[j].x), c2, acc[0], false);
                        acc[1] = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16, q[j].y), c2, acc[1], false);
                        acc[2] = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16, q[j].z), c2, acc[2], false);
                        acc[3] = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16, q[j].w), c2, acc[3], false);
                    }
                    if ((!CL && !lane_any) || (PP_ABLATE(a.debug) & 1)) continue;
                    constexpr int sh = OUTB == 8 ? 19 : 11 + 16 - OUTB;
                    constexpr int mx = (1 << OUTB) - 1;
                    if constexpr (FUSE == 0 && OUTB > 8 && PIXPATH_PACKED_CLAMP) {
                        if (CL || (lane_full && a.vec_dst)) {  // 16-bit samples, vector store: packed clamp
                            uint2 v;
                            v.x = clamp_pack16<sh, mx>(acc[0], acc[1]);
                            v.y = clamp_pack16<sh, mx>(acc[2], acc[3]);
                            *reinterpret_cast<uint2 *>(drow_p + 2 * vxo) = v;
                            __builtin_amdgcn_sched_barrier(0);
                            continue;
                        }
                    }
                    int o[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) o[j] = min(max(acc[j] >> sh, 0), mx);
                    if constexpr (FUSE >= 8) {
                        if (jfuse == 2) {  // into ring2 (second-stage input)
                            uint32_t bq[4];
#pragma unroll
                            for (int j = 0; j < 4; ++j) {  // opaque bytes (v_ashr_pk_u8_i32, see store4)
                                bq[j] = (uint32_t)o[j];
                                asm volatile("" : "+v"(bq[j]));
                            }
                            *reinterpret_cast<uint32_t *>(ring2b + (y & J.r2mask) * TW + vx) =
                                bq[0] | (bq[1] << 8) | (bq[2] << 16) | (bq[3] << 24);
                            __builtin_amdgcn_sched_barrier(0);
                            continue;
                        }
                        if (jfuse == 1) {  // identity second stage: one 4096 tap on x << 7
                            constexpr int r2 = OUT2 == 8 ? 64 << 12 : 1 << (10 + 16 - OUT2);
                            constexpr int s2 = OUT2 == 8 ? 19 : 11 + 16 - OUT2;
                            int w[4];
#pragma unroll
                            for (int j = 0; j < 4; ++j) w[j] = ((o[j] << 19) + r2) >> s2;
                            store4<OUT2>(drow_p, vxo, w, CL || (lane_full && a.vec_dst), jdw);
                            __builtin_amdgcn_sched_barrier(0);
                            continue;
                        }
                    }
                    if constexpr (FUSE == 1) {
                        uint8_t *pk = drow_p + J.pk_off;
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            if (xo + j < J.dw) pk[(xo + j) * J.pk_step] = (uint8_t)o[j];
                    } else {
                        store4<OUTB>(drow_p, vxo, o, CL || (lane_full && a.vec_dst), jdw);
                    }
                    // keep the next row's window reads behind this row's math
                    // (hoisting them all costs ~50 VGPRs and two waves/SIMD)
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        };
        auto vdispatch = [&](auto cl_c) {
            switch (vtp) {  // uniform, once per chunk; arms up to VTM only (register budget)
            case 1: vpass(std::integral_constant<int, 1>{}, cl_c); break;
            case 2: if constexpr (VTM >= 2) vpass(std::integral_constant<int, 2>{}, cl_c); break;
            case 3: if constexpr (VTM >= 3) vpass(std::integral_constant<int, 3>{}, cl_c); break;
            case 4: if constexpr (VTM >= 4) vpass(std::integral_constant<int, 4>{}, cl_c); break;
            case 5: if constexpr (VTM >= 5) vpass(std::integral_constant<int, 5>{}, cl_c); break;
            case 6: if constexpr (VTM >= 6) vpass(std::integral_constant<int, 6>{}, cl_c); break;
            case 7: if constexpr (VTM >= 7) vpass(std::integral_constant<int, 7>{}, cl_c); break;
            default: if constexpr (VTM >= 8) vpass(std::integral_constant<int, 8>{}, cl_c); break;
            }
        };
        if constexpr (FUSE == 9 || FUSE == 11) {
            // the host picks these instances only for clamped plans (every
            // plane's width a multiple of 4, vector stores): one copy of the loop
            vdispatch(std::true_type{});
        } else if constexpr (FUSE != 1 && strip_clamp_path<ST, OUTB, HW, VTM, FUSE>()) {
            if (clamp) vdispatch(std::true_type{});
            else vdispatch(std::false_type{});
        } else {
            vdispatch(std::false_type{});
        }
        if constexpr (FUSE >= 8 && FUSE != 9) {
            // ---- second stage (fuse 2): vertical filter of the ring2 rows ----
            if (jfuse == 2 && !(PP_ABLATE(a.debug) & 16)) {  // debug 16: no second stage (timing only)
                __syncthreads();  // this chunk's first-stage rows are in ring2
                const int lo2 = max(chunk2[4 * ci], r2lo), hi2 = min(chunk2[4 * ci + 1], r2hi);
                const kconst int32_t *vrow2 = as_kconst<int32_t>(J.vrow2);
                // rows in pairs (2m, 2m + 1): the vertical 4:2:0 -> 4:2:2 step is
                // a 2x upsample, so both rows of a pair read one window of ring2
                // rows (record [m][16]: base row, VT2 taps of row 2m, VT2 of
                // row 2m + 1, zero outside each row's own taps) -- the rows are
                // read and interleaved into v_dot2 pairs once for two output rows.
                // The records of G2 pairs come through the scalar cache at once.
                auto pass2 = [&](auto vt_c, auto cl_c) {
                    constexpr int VT2 = decltype(vt_c)::value;
                    constexpr bool CL = decltype(cl_c)::value;
                    const int vx = CL ? cxv : cx, vxo = CL ? xov : xo;
                    constexpr int G2 = 2;
                    const int m_lo = lo2 >> 1, m_hi = (hi2 + 1) >> 1;
                    for (int g0 = m_lo + rg; g0 < m_hi; g0 += 4 * G2) {
                        int vb[G2];
                        int32_t cf[G2][2][VT2];
#pragma unroll
                        for (int i = 0; i < G2; ++i) {
                            const kconst int32_t *row = vrow2 + (int64_t)min(g0 + 4 * i, m_hi - 1) * 16;
                            vb[i] = row[0];
#pragma unroll
                            for (int j = 0; j < VT2; ++j) {
                                cf[i][0][j] = row[1 + j];
                                cf[i][1][j] = row[1 + VT2 + j];
                            }
                        }
#pragma unroll
                        for (int i = 0; i < G2; ++i) {
                            const int m = g0 + 4 * i;
                            if (m >= m_hi) break;
                            // rows vb + 2j, vb + 2j + 1 from the byte ring, interleaved into
                            // the (row, row + 1) sample pairs of v_dot2; the first stage's
                            // << 7 (hScale8To15 of the identity H filter) moves onto the sum
                            uint32_t ra[VT2], rb[VT2];
#pragma unroll
                            for (int j = 0; j < VT2; ++j) {
                                ra[j] = *reinterpret_cast<const uint32_t *>(ring2b + ((vb[i] + 2 * j) & J.r2mask) * TW + vx);
                                rb[j] = *reinterpret_cast<const uint32_t *>(ring2b + ((vb[i] + 2 * j + 1) & J.r2mask) * TW + vx);
                            }
                            int acc2[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
                            for (int j = 0; j < VT2; ++j) {  // interleave once, accumulate both rows
                                const uint32_t q[4] = {__builtin_amdgcn_perm(rb[j], ra[j], 0x0c040c00u),
                                                       __builtin_amdgcn_perm(rb[j], ra[j], 0x0c050c01u),
                                                       __builtin_amdgcn_perm(rb[j], ra[j], 0x0c060c02u),
                                                       __builtin_amdgcn_perm(rb[j], ra[j], 0x0c070c03u)};
#pragma unroll
                                for (int h = 0; h < 2; ++h) {
                                    const v2i16 c2 = __builtin_bit_cast(v2i16, cf[i][h][j]);
#pragma unroll
                                    for (int e = 0; e < 4; ++e)
                                        acc2[h][e] = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16, q[e]), c2, acc2[h][e], false);
                                }
                            }
#pragma unroll
                            for (int h = 0; h < 2; ++h) {
                                const int r2 = 2 * m + h;
                                int acc[4];
#pragma unroll
                                for (int j = 0; j < 4; ++j)
                                    acc[j] = (acc2[h][j] << 7) + (OUT2 == 8 ? 64 << 12 : 1 << (10 + 16 - OUT2));
                                if ((!CL && !lane_any) || r2 >= hi2) continue;
                                constexpr int s2 = OUT2 == 8 ? 19 : 11 + 16 - OUT2;
                                if constexpr (FUSE == 11) {  // (FUSE 10 spills with it)
                                    if (CL || (lane_full && a.vec_dst)) {
                                        // (acc2 << 7) + 2^16 >> 17 == (acc2 + 512) >> 10, the high
                                        // half of 64 (acc2 + 512): one v_lshl_add per output, then
                                        // both halves' clamp as packed 16-bit ops (clamp_pack16)
                                        int hv[4];
#pragma unroll
                                        for (int j = 0; j < 4; ++j) hv[j] = (acc2[h][j] << 6) + 32768;
                                        uint2 v;
                                        v.x = clamp_pack16<16, 1023>(hv[0], hv[1]);
                                        v.y = clamp_pack16<16, 1023>(hv[2], hv[3]);
                                        *reinterpret_cast<uint2 *>(dbase + (int64_t)r2 * dls + 2 * vxo) = v;
                                        continue;
                                    }
                                }
                                int w[4];
#pragma unroll
                                for (int j = 0; j < 4; ++j) w[j] = min(max(acc[j] >> s2, 0), (1 << OUT2) - 1);
                                store4<OUT2>(dbase + (int64_t)r2 * dls, vxo, w, CL || (lane_full && a.vec_dst), jdw);
                            }
                            __builtin_amdgcn_sched_barrier(0);
                        }
                    }
                };
                auto dispatch2 = [&](auto cl_c) {
                    switch (J.vtp2) {  // uniform; the host allows <= 3 pairs (a row pair's window)
                    case 1: pass2(std::integral_constant<int, 1>{}, cl_c); break;
                    case 2: pass2(std::integral_constant<int, 2>{}, cl_c); break;
                    default: pass2(std::integral_constant<int, 3>{}, cl_c); break;
                    }
                };
                if constexpr (FUSE == 11) {
                    dispatch2(std::true_type{});
                } else if constexpr (strip_clamp_path<ST, OUTB, HW, VTM, FUSE>()) {
                    if (clamp) dispatch2(std::true_type{});
                    else dispatch2(std::false_type{});
                } else {
                    dispatch2(std::false_type{});
                }
            }
        }
        __builtin_amdgcn_s_setprio(0);
    }
}


inline int strip_vtm_bucket_impl(int vtp) { return vtp <= 2 ? 2 : vtp <= 3 ? 3 : vtp <= 5 ? 5 : 8; }

#define PP_STRIP_VTM(ST, OUTB, HW, FUSE, TW)                                 \
    switch (vtm) {                                                           \
    case 2: return strip_kernel<ST, OUTB, HW, 2, FUSE, TW>;                  \
    case 3: return strip_kernel<ST, OUTB, HW, 3, FUSE, TW>;                  \
    case 5: return strip_kernel<ST, OUTB, HW, 5, FUSE, TW>;                  \
    default: return strip_kernel<ST, OUTB, HW, 8, FUSE, TW>;                 \
    }
#define PP_STRIP_HW_FT(ST, OUTB, FUSE, TW)                                   \
    switch (hw) {                                                            \
    case 3: PP_STRIP_VTM(ST, OUTB, 3, FUSE, TW)                              \
    case 4: PP_STRIP_VTM(ST, OUTB, 4, FUSE, TW)                              \
    case 5: PP_STRIP_VTM(ST, OUTB, 5, FUSE, TW)                              \
    case 6: PP_STRIP_VTM(ST, OUTB, 6, FUSE, TW)                              \
    case 8: PP_STRIP_VTM(ST, OUTB, 8, FUSE, TW)                              \
    case 10: PP_STRIP_VTM(ST, OUTB, 10, FUSE, TW)                            \
    case 12: PP_STRIP_VTM(ST, OUTB, 12, FUSE, TW)                            \
    case 16: PP_STRIP_VTM(ST, OUTB, 16, FUSE, TW)                            \
    default: return nullptr;                                                 \
    }
#define PP_STRIP_HW_F(ST, OUTB, FUSE) PP_STRIP_HW_FT(ST, OUTB, FUSE, 256)
// 512-column strips are reachable only through the PIXPATH_STRIP_TW knob of
// the measurement build (scale.hip plan_create), so only it instantiates them
#ifdef PIXPATH_ABLATE
#define PP_STRIP_HW(ST, OUTB)                                                \
    if (tw == 512) {                                                         \
        PP_STRIP_HW_FT(ST, OUTB, 0, 512)                                     \
    }                                                                        \
    PP_STRIP_HW_FT(ST, OUTB, 0, 256)
#else
#define PP_STRIP_HW(ST, OUTB)                                                \
    (void)tw;                                                                \
    PP_STRIP_HW_FT(ST, OUTB, 0, 256)
#endif

}  // namespace pp
