// Scaler plans and the fused separable polyphase kernel (gfx950).
//
// Reference semantics: FFmpeg 7.0 libswscale generic path as used by
// `scale=W:H:flags=bicubic` (lib/ffmpeg.py:992, :1038, :1213, :800) and the
// implicit `-pix_fmt` conversions (:994, :1048, :1198):
//   hScale{8,16}To15   -> 15-bit intermediates  (Σ src*hcoef) >> (8-bit: 7, N-bit: N-1), min 32767
//   yuv2planeX_8       -> clip_u8((dither<<12 + Σ inter*vcoef) >> 19)
//   yuv2planeX_10      -> clip_u10((1<<16 + Σ inter*vcoef) >> 17)
// dither = ff_dither_8x8_128[row & 7][(col + off) & 7] when a >8-bit source is
// narrowed to 8 bit (off = 3 for the V plane), flat 64 otherwise.
//
// MI355X design ("strip streaming"): one workgroup (256 lanes = 4 wave64) owns
// a TW-wide (256 unless a large downscale needs narrower) column strip of one
// plane of one frame, split vertically into a few segments, and walks it top to
// bottom in chunks of CHO output rows.  Per chunk it stages only the source
// rows not seen before (16-B vector loads -> LDS), runs the horizontal pass
// LDS->LDS into a ring of 15-bit intermediate rows (coefficients in VGPRs, one
// output column per lane), then the vertical pass ring->HBM with wave-uniform
// coefficients (scalar loads) and 4 outputs per lane (one ds_read_b64 per tap).
// Every source row is read from HBM once per strip (plus a few rows at segment
// seams and a column halo of ~taps/TW), intermediates never touch HBM, and all
// three planes of a whole frame batch go in ONE launch
// (blockIdx.x = strip x segment over the planes, blockIdx.y = frame).
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <type_traits>

#include "filters.hpp"
#include "scale_dev.hpp"

namespace pp {

// TWC: 256 when every plane uses 256-column strips (the usual case: lane =
// column, wave = row group, all row loops wave-uniform), 0 for the general
// strip width.
template <typename ST, int OUTB, int HT, int TWC>
__global__ __launch_bounds__(kThreads) void scale_kernel(const ScaleArgs a) {
    extern __shared__ __align__(16) uint16_t lds[];
    // 1-D grid of frames x tiles, XCD-aware: an XCD walks consecutive strips of
    // consecutive frames, so strip and segment halos hit its L2
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int frame = L / a.tiles;
    int t = L - frame * a.tiles;
    int p = 0;
    if (a.nplanes > 1 && t >= a.pl[1].tile_base) p = 1;
    if (a.nplanes > 2 && t >= a.pl[2].tile_base) p = 2;
    const PlaneJob &J = a.pl[p];
    t -= J.tile_base;
    const int seg = t / J.tiles_x, tx = t - seg * J.tiles_x;
    const int TW = TWC ? TWC : J.tw;
    const int x0 = tx * TW, nx = min(TW, J.dw - x0);
    const int c0 = J.tile_c0[tx], cn = J.tile_cn[tx];
    const int S = J.S;
    uint16_t *src_t = lds;                                              // [maxnew][S]
    // window of 15-bit intermediates, row pairs interleaved per column: the
    // dword [k][c] holds rows (base + 2k, base + 2k + 1) of column c, base = the
    // chunk's first source row rounded down to even (rows a chunk shares with
    // the previous one are moved down at the chunk start, so reads never wrap)
    int16_t *ring = reinterpret_cast<int16_t *>(lds + J.maxnew * S);
    uint32_t *win = reinterpret_cast<uint32_t *>(ring);
    int32_t *vcl = reinterpret_cast<int32_t *>(ring + J.ring * TW);     // [cho][vtp] chunk V tap pairs
    int32_t *vpl = vcl + J.cho * J.vtp;                                  // [cho] chunk V base rows
    const int tid = threadIdx.x;
    const ST *sbase = reinterpret_cast<const ST *>(a.src[p] + frame * a.sfs[p]);
    uint8_t *dbase = a.dst[p] + frame * a.dfs[p];

    // horizontal-pass lane mapping: one output column per lane, r_step rows at a time
    const int col = TWC ? tid : tid % TW, r_first = TWC ? 0 : tid / TW, r_step = TWC ? 1 : kThreads / TW;
    // taps as packed 16-bit pairs for v_dot2_i32_i16 (HT is 1 or even)
    constexpr int HP = HT == 1 ? 1 : HT / 2;
    v2i16 hcp[HP];
#pragma unroll
    for (int j = 0; j < HP; ++j) hcp[j] = v2i16{0, 0};
    int hbias = 0;  // 32768 * sum(coef): undoes the staging bias of 16-bit samples
    int hoff = 0;
    if (col < nx) {
        const int x = x0 + col;
        hoff = J.hpos[x] - c0;
        int hsum = 0;
        if constexpr (HT == 1) {
            const int c = J.hcoef[x];
            hcp[0] = v2i16{(int16_t)c, 0};
            hsum = c;
        } else {
#pragma unroll
            for (int j = 0; j < HP; ++j) {
                const int16_t c0_ = J.hcoef[(int64_t)x * HT + 2 * j], c1_ = J.hcoef[(int64_t)x * HT + 2 * j + 1];
                hcp[j] = v2i16{c0_, c1_};
                hsum += c0_ + c1_;
            }
        }
        if constexpr (sizeof(ST) == 2) hbias = hsum * 32768;
    }
    // vertical-pass lane mapping: 4 adjacent outputs per lane
    const int groups = TW / 4;
    const int lane_g = TWC ? (tid & 63) : tid % groups, row_first = TWC ? (tid >> 6) : tid / groups,
              row_step = TWC ? 4 : kThreads / groups;
    const int cx = lane_g * 4;
    const int vtp = J.vtp;
    (void)J.twl;

    const int y_begin = seg * J.seg_h, y_end = min(J.dh, y_begin + J.seg_h);
    constexpr int CH = 16 / sizeof(ST);
    const int cpr = (cn + CH - 1) / CH;  // 16-B chunks per staged row
    const int64_t sls = a.sls[p];
    const bool vec = a.vec_src;
    const int sw = J.sw;
    // a 16-B load that straddles num_records reads 0 as a whole, so the last
    // row counts up to its 16-B-rounded width (inside the pitch: the vector
    // path requires 16-B aligned linesizes; see pp_frames in pixpath.h)
    const int64_t last_row = std::min<int64_t>(sls, ((int64_t)sw * sizeof(ST) + 15) & ~int64_t(15));
    const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(sbase, (int)((int64_t)(J.sh - 1) * sls + last_row));
    const int cbyte = c0 * (int)sizeof(ST);
    // byte offset of chunk `id` of rows [from, ...) (kOobOff when id >= total)
    auto chunk_off = [&](int id, int from, int total) {
        const int r = id / cpr, ch = id - r * cpr;
        const int off = (from + r) * (int)sls + cbyte + ch * 16;
        return id < total ? off : kOobOff;
    };
    // staging coordinates, fixed per lane when a row has <= 256 chunks: chunk
    // column s_ch of rows s_r0, s_r0 + s_rstep, ... (no division per chunk)
    const bool fixed = cpr <= kThreads;
    const int s_rstep = fixed ? kThreads / cpr : 1;
    const int s_r0 = fixed ? tid / cpr : 0, s_ch = fixed ? tid - s_r0 * cpr : 0;
    const bool s_on = fixed && s_r0 < s_rstep;
    const int s_lds = s_r0 * S + s_ch * CH;            // LDS sample offset of the lane's first row
    const int s_goff = s_r0 * (int)sls + cbyte + s_ch * 16;  // its byte offset within the plane, less `from` rows
    // issue the loads of chunk rows [from, hi) for this lane (first kPF rows of
    // its column); straight-line code, so the kPF loads are all in flight at once
    auto prefetch = [&](Prefetch<ST> &pf, int from, int hi_) {
        if (!vec) return;
        if (fixed) {
            const int nrow = hi_ - from;
#pragma unroll
            for (int k = 0; k < kPF; ++k) {
                const int r = s_r0 + k * s_rstep;
                pf.v[k] = bload16(rs, (s_on && r < nrow) ? s_goff + (from + k * s_rstep) * (int)sls : kOobOff);
            }
        } else {
            const int total = (hi_ - from) * cpr;
#pragma unroll
            for (int k = 0; k < kPF; ++k) pf.v[k] = bload16(rs, chunk_off(tid + k * kThreads, from, total));
        }
    };
    // write the prefetched chunks to LDS and stage any remainder synchronously
    auto commit = [&](const Prefetch<ST> &pf, int from, int hi_) {
        const int total = (hi_ - from) * cpr;
        if (!vec) {
            for (int id = tid; id < total; id += kThreads) {
                const int r = id / cpr, ch = id - r * cpr;
                const ST *g = reinterpret_cast<const ST *>(reinterpret_cast<const uint8_t *>(sbase) +
                                                           (int64_t)(from + r) * sls);
                store16<ST>(src_t + r * S + ch * CH, load16_scalar<ST>(g, c0 + ch * CH, sw));
            }
            return;
        }
        if (fixed) {
            const int nrow = hi_ - from;
            if (!s_on) return;
#pragma unroll
            for (int k = 0; k < kPF; ++k)
                if (s_r0 + k * s_rstep < nrow) store16<ST>(src_t + s_lds + k * s_rstep * S, pf.v[k]);
            for (int k = kPF; s_r0 + k * s_rstep < nrow; ++k)
                store16<ST>(src_t + s_lds + k * s_rstep * S, bload16(rs, s_goff + (from + k * s_rstep) * (int)sls));
            return;
        }
#pragma unroll
        for (int k = 0; k < kPF; ++k) {
            const int id = tid + k * kThreads;
            if (id < total) {
                const int r = id / cpr, ch = id - r * cpr;
                store16<ST>(src_t + r * S + ch * CH, pf.v[k]);
            }
        }
        for (int id = tid + kPF * kThreads; id < total; id += kThreads) {
            const int r = id / cpr, ch = id - r * cpr;
            store16<ST>(src_t + r * S + ch * CH, bload16(rs, chunk_off(id, from, total)));
        }
    };

    int next_src = J.chunk_lo[y_begin / J.cho];
    int base = next_src & ~1;  // window row 0 (even source row)
    Prefetch<ST> pf;
    // rows the first chunk needs
    int pf_from = next_src, pf_hi = J.chunk_hi[y_begin / J.cho];
    if (pf_from < J.chunk_lo[y_begin / J.cho]) pf_from = J.chunk_lo[y_begin / J.cho];
    prefetch(pf, pf_from, pf_hi);
    // one H-pass output row: taps over the staged source row at `sp` (window
    // start hoff, 4-B aligned reads, odd starts re-paired with v_alignbit)
    const int odd = hoff & 1;
    const uint32_t ash = odd * 16;
    auto hrow = [&](const uint16_t *sp) -> uint32_t {
        int acc;
        if constexpr (HT == 1) {
            acc = hbias + static_cast<int>(static_cast<int16_t>(sp[odd])) * hcp[0][0];
        } else {
            const uint32_t *sw32 = static_cast<const uint32_t *>(__builtin_assume_aligned(sp, 4));
            uint32_t w[HP + 1];
#pragma unroll
            for (int j = 0; j <= HP; ++j) w[j] = sw32[j];
            acc = dot2_acc(__builtin_bit_cast(v2i16, __builtin_amdgcn_alignbit(w[1], w[0], ash)), hcp[0], hbias);
#pragma unroll
            for (int j = 1; j < HP; ++j)
                acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16, __builtin_amdgcn_alignbit(w[j + 1], w[j], ash)),
                                             hcp[j], acc, false);
        }
        acc >>= a.hshift;
        return static_cast<uint32_t>(acc < 32767 ? acc : 32767) & 0xffffu;
    };
    const int nxw = TWC ? TW : nx;  // window columns written (TWC: all, harmlessly)
    for (int y0 = y_begin; y0 < y_end; y0 += J.cho) {
        const int ci = y0 / J.cho;
        const int lo = J.chunk_lo[ci], hi = J.chunk_hi[ci];
        if (next_src < lo) next_src = lo;
        const int nnew = hi - next_src;
        const int nbase = lo & ~1;
        // rows kept from the previous chunk: [nbase, next_src), as whole pairs
        const int keep = next_src > nbase ? (next_src - nbase + 1) >> 1 : 0;
        const int shift = (nbase - base) >> 1;
        // ---- commit the prefetched rows (src_t is not read by the vertical pass) ----
        if (nnew > 0) commit(pf, next_src, hi);
        __syncthreads();  // staged rows visible; every wave has left the previous vertical pass
        // ---- this chunk's vertical taps/rows: written only after the barrier above
        // (the previous vertical pass reads them), visible after the one below ----
        {
            const int ny_c = min(J.cho, y_end - y0);
            for (int i = tid; i < ny_c * vtp; i += kThreads) vcl[i] = J.vcoef2[(int64_t)y0 * vtp + i];
            for (int i = tid; i < ny_c; i += kThreads) vpl[i] = J.vbase[y0 + i] - nbase;
        }
        // ---- move the kept pairs down to the window start: each column by one
        // lane, in increasing order, so no lane reads a slot already overwritten ----
        if (shift > 0 && r_first == 0 && col < nxw) {
            for (int k = 0; k < keep; ++k) win[k * TW + col] = win[(k + shift) * TW + col];
        }
        // general strip width: other lanes of the column write new pairs that the
        // copy may still have to read (TWC: one lane per column, program order)
        if constexpr (!TWC) __syncthreads();
        base = nbase;
        // ---- horizontal pass into the window, one row pair per step -------------
        // (TWC: lanes past the strip's last column compute with zero taps and
        // write window columns the vertical pass never reads -- no divergence)
        if (nnew > 0 && col < nxw) {
            const int i0 = next_src - base;            // window row of the first new row
            const uint16_t *sp = src_t + hoff - odd;
            // a half pair at each end (its other row is kept, or not needed), full
            // pairs in between: one packed 32-bit write per two rows
            const int kf0 = (i0 + 1) >> 1, kf1 = (i0 + nnew) >> 1;
            if ((i0 & 1) && r_first == 0)  // high row of pair i0/2 (same lane as the copy above)
                reinterpret_cast<uint16_t *>(win + (i0 >> 1) * TW + col)[1] = static_cast<uint16_t>(hrow(sp));
            if (((i0 + nnew) & 1) && r_first == r_step - 1)  // low row of the last pair
                reinterpret_cast<uint16_t *>(win + kf1 * TW + col)[0] =
                    static_cast<uint16_t>(hrow(sp + (nnew - 1) * S));
            for (int k = kf0 + r_first; k < kf1; k += r_step) {
                const int ra = 2 * k - i0;             // new-row index of the pair's low row
                const uint32_t lo16 = hrow(sp + ra * S), hi16 = hrow(sp + (ra + 1) * S);
                win[k * TW + col] = lo16 | (hi16 << 16);
            }
        }
        if (nnew > 0) next_src = hi;
        __syncthreads();
        // ---- prefetch the next chunk's new rows; their loads overlap the V pass ----
        if (y0 + J.cho < y_end) {
            const int nlo = J.chunk_lo[ci + 1], nhi = J.chunk_hi[ci + 1];
            prefetch(pf, max(next_src, nlo), nhi);
        }
        // ---- vertical pass: output rows [y0, y0 + cho) --------------------------
        const int ny = min(J.cho, y_end - y0);
        for (int yy0 = row_first; yy0 < ny + row_first; yy0 += row_step) {
            int yy = yy0;
            if (TW == kTileW) yy = __builtin_amdgcn_readfirstlane(yy);
            if (yy >= ny) break;
            const int y = y0 + yy;
            const int32_t *vc = vcl + yy * vtp;
            if (cx >= nx) continue;
            int acc0 = 0, acc1 = 0, acc2 = 0, acc3 = 0;
            // pairs (vbase + 2j, vbase + 2j + 1) of columns cx..cx+3: one 16-B read each
            const uint4 *rp = reinterpret_cast<const uint4 *>(win + (vpl[yy] >> 1) * TW + cx);
#pragma unroll 2
            for (int j = 0; j < vtp; ++j) {
                const v2i16 cf = __builtin_bit_cast(v2i16, vc[j]);
                const uint4 q = rp[j * (TW / 4)];
                acc0 = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16, q.x), cf, acc0, false);
                acc1 = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16, q.y), cf, acc1, false);
                acc2 = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16, q.z), cf, acc2, false);
                acc3 = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16, q.w), cf, acc3, false);
            }
            const int x = x0 + cx;
            int o[4];
            if constexpr (OUTB == 8) {
                const int drow = y & 7;
                int d[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) d[j] = a.dither ? c_dither[drow][(x + j + J.dither_off) & 7] : 64;
                o[0] = (acc0 + (d[0] << 12)) >> 19;
                o[1] = (acc1 + (d[1] << 12)) >> 19;
                o[2] = (acc2 + (d[2] << 12)) >> 19;
                o[3] = (acc3 + (d[3] << 12)) >> 19;
#pragma unroll
                for (int j = 0; j < 4; ++j) o[j] = min(max(o[j], 0), 255);
                uint8_t *drow_p = dbase + (int64_t)y * a.dls[p];
                if (a.vec_dst && x + 3 < J.dw) {
                    *reinterpret_cast<uint32_t *>(drow_p + x) =
                        (uint32_t)o[0] | ((uint32_t)o[1] << 8) | ((uint32_t)o[2] << 16) | ((uint32_t)o[3] << 24);
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (x + j < J.dw) drow_p[x + j] = (uint8_t)o[j];
                }
            } else {
                constexpr int sh = 11 + 16 - OUTB;
                constexpr int mx = (1 << OUTB) - 1;
                o[0] = (acc0 + (1 << (sh - 1))) >> sh;
                o[1] = (acc1 + (1 << (sh - 1))) >> sh;
                o[2] = (acc2 + (1 << (sh - 1))) >> sh;
                o[3] = (acc3 + (1 << (sh - 1))) >> sh;
#pragma unroll
                for (int j = 0; j < 4; ++j) o[j] = min(max(o[j], 0), mx);
                uint16_t *drow_p = reinterpret_cast<uint16_t *>(dbase + (int64_t)y * a.dls[p]);
                if (a.vec_dst && x + 3 < J.dw) {
                    uint2 v;
                    v.x = (uint32_t)o[0] | ((uint32_t)o[1] << 16);
                    v.y = (uint32_t)o[2] | ((uint32_t)o[3] << 16);
                    *reinterpret_cast<uint2 *>(drow_p + x) = v;
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (x + j < J.dw) drow_p[x + j] = (uint16_t)o[j];
                }
            }
        }
    }
}

// planarCopyWrapper (same subsampling, same or wider depth): 8 samples per lane.
__global__ __launch_bounds__(256) void copy_widen_kernel(const uint8_t *src, int64_t sls, int64_t sfs, int sbytes,
                                                         uint8_t *dst, int64_t dls, int64_t dfs, int dbytes,
                                                         int w, int h, int shift) {
    const int frame = blockIdx.z;
    const int y = blockIdx.y;
    const uint8_t *s = src + frame * sfs + (int64_t)y * sls;
    uint8_t *d = dst + frame * dfs + (int64_t)y * dls;
    for (int x = (blockIdx.x * 256 + threadIdx.x) * 8; x < w; x += gridDim.x * 256 * 8) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            if (x + e >= w) break;
            const int v = sbytes == 1 ? s[x + e] : reinterpret_cast<const uint16_t *>(s)[x + e];
            if (dbytes == 1)
                d[x + e] = (uint8_t)v;
            else
                reinterpret_cast<uint16_t *>(d)[x + e] = (uint16_t)(v << shift);
        }
    }
}

// yuv422pToUyvyWrapper: interleave U Y V Y (8-bit); one lane writes 16 bytes.
__global__ __launch_bounds__(256) void interleave_uyvy_kernel(const uint8_t *Y, const uint8_t *U, const uint8_t *V,
                                                              int64_t yls, int64_t uls, int64_t vls, int64_t yfs,
                                                              int64_t ufs, int64_t vfs, uint8_t *dst, int64_t dls,
                                                              int64_t dfs, int w, int h) {
    const int frame = blockIdx.z, y = blockIdx.y;
    const uint8_t *yr = Y + frame * yfs + (int64_t)y * yls;
    const uint8_t *ur = U + frame * ufs + (int64_t)y * uls;
    const uint8_t *vr = V + frame * vfs + (int64_t)y * vls;
    uint8_t *d = dst + frame * dfs + (int64_t)y * dls;
    const int pairs = (w + 1) / 2;
    for (int q = (blockIdx.x * 256 + threadIdx.x) * 4; q < pairs; q += gridDim.x * 256 * 4) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int i = q + e;
            if (i >= pairs) break;
            d[4 * i + 0] = ur[i];
            d[4 * i + 1] = yr[2 * i];
            d[4 * i + 2] = vr[i];
            d[4 * i + 3] = (2 * i + 1 < w) ? yr[2 * i + 1] : 0;
        }
    }
}


template <typename ST, int OUTB, int TWC>
KernelFn pick_ht_tw(int ht) {
    switch (ht) {
    case 1: return scale_kernel<ST, OUTB, 1, TWC>;
    case 2: return scale_kernel<ST, OUTB, 2, TWC>;
    case 4: return scale_kernel<ST, OUTB, 4, TWC>;
    case 6: return scale_kernel<ST, OUTB, 6, TWC>;
    case 8: return scale_kernel<ST, OUTB, 8, TWC>;
    case 12: return scale_kernel<ST, OUTB, 12, TWC>;
    case 16: return scale_kernel<ST, OUTB, 16, TWC>;
    case 24: return scale_kernel<ST, OUTB, 24, TWC>;
    case 32: return scale_kernel<ST, OUTB, 32, TWC>;
    default: return nullptr;
    }
}

template <typename ST, int OUTB>
KernelFn pick_ht(int ht, bool tw256) {
    return tw256 ? pick_ht_tw<ST, OUTB, kTileW>(ht) : pick_ht_tw<ST, OUTB, 0>(ht);
}

inline int ht_bucket(int t) {
    static const int b[] = {1, 2, 4, 6, 8, 12, 16, 24, 32};
    for (int v : b)
        if (t <= v) return v;
    return -1;
}

} // namespace pp

// ---------------------------------------------------------------------------
struct pp_scale_plan {
    enum Kind { GENERIC, COPY, INTERLEAVE, GENERIC_UYVY, CHAIN } kind = GENERIC;
    pp_ctx *ctx = nullptr;
    int src_fmt = 0, dst_fmt = 0, sw = 0, sh = 0, dw = 0, dh = 0;
    pp::FmtInfo si{}, di{};
    int csw = 0, csh = 0, cdw = 0, cdh = 0;
    pp::FilterBank f[4];   // hl, hc, vl, vc (FFmpeg layout)
    int ht = 1;            // compiled H-tap bucket
    pp::PlaneJob job[3]{};
    void *dev = nullptr;   // all tables in one allocation
    void *scratch = nullptr; int64_t scratch_plane[3] = {0, 0, 0}; // GENERIC_UYVY planar 4:2:2 temp
    int scratch_frames = 0;
    size_t lds_bytes = 0;
    pp::PlaneJob fjob[3]{}; // strip_kernel jobs (fast_hw > 0)
    int fast_hw = 0;        // H window dwords of strip_kernel, 0 = generic kernel only
    size_t fast_lds = 0;
    int fast_tw = 256;      // strip_kernel strip width = threads per workgroup (256 or 512)
    int fast_tiles = 0;     // strip_kernel workgroups per frame (all planes)
    // CHAIN (pp_scale_chain_plan_create): this plan is the first stage (-> yuv420p)
    pp_scale_plan *stage2 = nullptr;  // yuv420p -> target at the same size (two-launch path)
    int chain_out = 0;                // target bit depth
    Kind first_kind = GENERIC;        // the first stage's own kind (two-launch path)
    bool chain_fused = false;         // one strip_kernel launch does both stages
    size_t chain_lds = 0;             // the fused launch's LDS (with `luma`: the chroma launch's)
    void *dev2 = nullptr;             // second-stage tables (vrow2, chunk2)
    // CHAIN, fused, 4:2:0 -> 4:2:2 target: luma's second stage is an identity
    // bank, so luma runs as its own launch of this first-stage plan (config-2
    // tiling: 32-row chunks, no second-stage ring) and the chain launch keeps
    // the chroma planes only -- LDS is sized per launch, so luma no longer
    // takes the 16-row chunks and ring2 LDS the chroma planes need
    pp_scale_plan *luma = nullptr;
    size_t fast_lds_plane[2] = {0, 0};  // strip_kernel LDS of the luma / chroma jobs alone
    bool direct = false;                // strip_kernel DIRECT tiling (8-bit source, HW 8): fast_lds = the V ring only
    std::vector<int32_t> chroma_lo, chroma_hi;  // chain first stage: source rows of each chroma chunk (host copy)
    hipStream_t side = nullptr;       // CHAIN with `luma`: the luma launch's stream when the two launches overlap
    hipEvent_t fork = nullptr, join = nullptr;
};

namespace {

using pp::FilterBank;

struct HostPlane {
    FilterBank::Compact h, v;
    std::vector<int32_t> c0, cn, lo, hi;
    std::vector<int32_t> vbase, vcoef2;  // V window as even-aligned row pairs
    int vtp = 1;
    int tiles_x = 0, nseg = 0, tw = 0, seg_h = 0, cho = 0, ring = 0, maxnew = 0, S = 0;
    // strip_kernel layout (its own strip width f_tw: column windows f_c0 / f_cn)
    std::vector<int32_t> hbase4, hcoefw, vrow16, f_c0, f_cn;
    int hw_need = 0, max_base = 0, S_fast = 0, f_tw = 256, f_tiles_x = 0, f_S = 0;
};

// Vertical taps regrouped as row pairs starting at an even row (the ring keeps
// row pairs interleaved, so one 32-bit LDS word is a v_dot2 operand).  An odd
// window start gets a leading zero tap; trailing zeros are dropped.
void pair_rows(HostPlane &hp) {
    const auto &v = hp.v;
    const int n = (int)v.pos.size();
    int vtp = 1;
    for (int i = 0; i < n; ++i) {
        int last = 0;
        for (int k = 0; k < v.taps; ++k)
            if (v.coef[(size_t)i * v.taps + k]) last = k;
        vtp = std::max(vtp, ((v.pos[i] & 1) + last + 2) / 2);
    }
    hp.vtp = vtp;
    hp.vbase.assign(n, 0);
    hp.vcoef2.assign((size_t)n * vtp, 0);
    for (int i = 0; i < n; ++i) {
        const int odd = v.pos[i] & 1;
        hp.vbase[i] = v.pos[i] - odd;
        auto tap = [&](int k) -> uint16_t {
            return (k >= 0 && k < v.taps) ? (uint16_t)v.coef[(size_t)i * v.taps + k] : 0;
        };
        for (int j = 0; j < vtp; ++j)
            hp.vcoef2[(size_t)i * vtp + j] =
                (int32_t)((uint32_t)tap(2 * j - odd) | ((uint32_t)tap(2 * j + 1 - odd) << 16));
    }
}

// Column window of every strip for a strip width.
int col_windows(HostPlane &hp, int sw, int dw, int tw) {
    const int tiles_x = (dw + tw - 1) / tw;
    hp.c0.assign(tiles_x, 0);
    hp.cn.assign(tiles_x, 0);
    int S = 0;
    for (int tx = 0; tx < tiles_x; ++tx) {
        int lo = sw, hi = 0;
        for (int x = tx * tw; x < std::min(dw, (tx + 1) * tw); ++x) {
            lo = std::min(lo, hp.h.pos[x]);
            hi = std::max(hi, hp.h.pos[x] + hp.h.taps);
        }
        lo &= ~15;
        const int n = (hi - lo + 15) & ~15;
        hp.c0[tx] = lo;
        hp.cn[tx] = n;
        S = std::max(S, n);
    }
    return S;
}

// Row windows per chunk of `cho` output rows; returns (max new rows per chunk, ring rows).
void row_chunks(HostPlane &hp, int sh, int dh, int cho, int seg_h, int *maxnew, int *ring) {
    const int nch = (dh + cho - 1) / cho;
    hp.lo.assign(nch, 0);
    hp.hi.assign(nch, 0);
    int span = 1;
    for (int ci = 0; ci < nch; ++ci) {
        int lo = sh, hi = 0;
        for (int y = ci * cho; y < std::min(dh, (ci + 1) * cho); ++y) {
            lo = std::min(lo, hp.v.pos[y]);
            hi = std::max(hi, hp.v.pos[y] + hp.v.taps);
        }
        hp.lo[ci] = lo;
        hp.hi[ci] = hi;
        span = std::max(span, hi - lo);
    }
    // simulate the kernel's walk to size the staging buffer
    int mn = 0;
    for (int y0 = 0; y0 < dh; y0 += seg_h) {
        int next = hp.lo[y0 / cho];
        for (int y = y0; y < std::min(dh, y0 + seg_h); y += cho) {
            const int ci = y / cho;
            if (next < hp.lo[ci]) next = hp.lo[ci];
            mn = std::max(mn, hp.hi[ci] - next);
            next = std::max(next, hp.hi[ci]);
        }
    }
    // window rows: from the chunk's even base to its last staged row or the
    // last row pair its vertical taps read (zero-weight taps included)
    int wr = 2;
    for (int ci = 0; ci < nch; ++ci) {
        const int b = hp.lo[ci] & ~1;
        int top = hp.hi[ci];
        for (int y = ci * cho; y < std::min(dh, (ci + 1) * cho); ++y) top = std::max(top, hp.vbase[y] + 2 * hp.vtp);
        wr = std::max(wr, top - b);
    }
    (void)span;
    *maxnew = std::max(mn, 1);
    *ring = (wr + 1) & ~1;
}

// LDS budget per workgroup in bytes (PIXPATH_SCALE_LDS_KB overrides, measurement only)
static size_t lds_budget() {
    const char *e = PP_KNOB("PIXPATH_SCALE_LDS_KB");
    return e ? (size_t)std::max(8, std::min(160, atoi(e))) * 1024 : (size_t)pp::kLdsBudget;
}

// Strip width / chunk height / segments for one plane: the widest strip and
// tallest chunk whose LDS (staging + ring) fits the budget; ~256-row segments.
int plan_tiles(HostPlane &hp, int sw, int sh, int dw, int dh, size_t *lds, std::string *err, int seg_force = 0,
               int cho_force = 0, bool ring_only = false) {
    static const int tws[] = {256, 128, 64, 32};
    static const int chos[] = {64, 48, 32, 24, 16, 8, 4, 2, 1};
    // tuning overrides (measurement only): tallest chunk, rows per segment
    const char *e_cho = PP_KNOB("PIXPATH_SCALE_CHO_MAX"), *e_seg = PP_KNOB("PIXPATH_SCALE_SEG_ROWS");
    const int cho_max = e_cho ? std::max(1, atoi(e_cho)) : cho_force > 0 ? cho_force : pp::kChoMax;
    const int seg_rows = seg_force > 0 ? seg_force : e_seg ? std::max(1, atoi(e_seg)) : pp::kSegRows;
    for (int tw : tws) {
        if (tw > 32 && tw / 2 >= dw) continue;  // narrower strips suffice for this plane
        const int S = col_windows(hp, sw, dw, tw);
        for (int cho : chos) {
            if (cho > cho_max) continue;
            int nseg = std::max(1, (dh + seg_rows / 2) / seg_rows);
            int seg_h = (dh + nseg - 1) / nseg;
            seg_h = (seg_h + cho - 1) / cho * cho;
            nseg = (dh + seg_h - 1) / seg_h;
            int maxnew, ring;
            row_chunks(hp, sh, dh, cho, seg_h, &maxnew, &ring);
            // ring_only: strip_kernel DIRECT, whose LDS is the V window ring alone
            const size_t bytes = ring_only ? (size_t)ring * tw * 2
                                           : (size_t)maxnew * S * 2 + (size_t)ring * tw * 2 + (size_t)cho * hp.vtp * 4 +
                                                 (size_t)cho * 4;
            if (bytes > lds_budget()) continue;
            hp.tiles_x = (dw + tw - 1) / tw;
            hp.nseg = nseg; hp.tw = tw; hp.seg_h = seg_h; hp.cho = cho;
            hp.ring = ring; hp.maxnew = maxnew; hp.S = S;
            *lds = std::max(*lds, bytes);
            return 0;
        }
    }
    *err = "scale ratio too large for the LDS budget";
    return -1;
}

// strip_kernel column windows for its strip width tw (256 or 512)
void fast_tiling(HostPlane &hp, int sw, int dw, int tw) {
    std::vector<int32_t> c0 = hp.c0, cn = hp.cn;  // the generic tiling's, kept
    hp.f_S = col_windows(hp, sw, dw, tw);
    hp.f_c0.swap(hp.c0);
    hp.f_cn.swap(hp.cn);
    hp.c0.swap(c0);
    hp.cn.swap(cn);
    hp.f_tw = tw;
    hp.f_tiles_x = (dw + tw - 1) / tw;
}

// strip_kernel windows: per 4-column lane group, an 8-B aligned base in the
// staged row and the dwords that hold every non-zero tap of its 4 outputs.
void fast_windows(HostPlane &hp, int dw) {
    const int taps = hp.h.taps, gpt = hp.f_tw / 4;
    hp.hbase4.assign((size_t)hp.f_tiles_x * gpt, 0);
    hp.hw_need = 1;
    hp.max_base = 0;
    for (int tx = 0; tx < hp.f_tiles_x; ++tx)
        for (int g = 0; g < gpt; ++g) {
            int lo = INT32_MAX, end = 0;
            for (int j = 0; j < 4; ++j) {
                const int x = tx * hp.f_tw + 4 * g + j;
                if (x >= dw) break;
                const int16_t *c = &hp.h.coef[(size_t)x * taps];
                for (int k = 0; k < taps; ++k)
                    if (c[k]) {
                        lo = std::min(lo, hp.h.pos[x] + k);
                        end = std::max(end, hp.h.pos[x] + k + 1);
                    }
            }
            if (lo == INT32_MAX) continue;
            const int base = (lo - hp.f_c0[tx]) & ~3;
            hp.hbase4[(size_t)tx * gpt + g] = base;
            hp.hw_need = std::max(hp.hw_need, (end - hp.f_c0[tx] - base + 1) / 2);
            hp.max_base = std::max(hp.max_base, base);
        }
}

// Taps of every output re-laid over its lane group's HW dwords (zero elsewhere).
void fast_coefs(HostPlane &hp, int dw, int HW) {
    const int taps = hp.h.taps, gpt = hp.f_tw / 4;
    hp.hcoefw.assign((size_t)hp.f_tiles_x * gpt * 4 * HW, 0);
    uint16_t *h16 = reinterpret_cast<uint16_t *>(hp.hcoefw.data());
    for (int tx = 0; tx < hp.f_tiles_x; ++tx)
        for (int g = 0; g < gpt; ++g)
            for (int j = 0; j < 4; ++j) {
                const int x = tx * hp.f_tw + 4 * g + j;
                if (x >= dw) break;
                const int base = hp.hbase4[(size_t)tx * gpt + g];
                for (int k = 0; k < taps; ++k) {
                    const int16_t c = hp.h.coef[(size_t)x * taps + k];
                    if (!c) continue;
                    const int s = hp.h.pos[x] + k - hp.f_c0[tx] - base;  // in [0, 2*HW)
                    h16[(((size_t)tx * gpt + g) * 4 + j) * HW * 2 + s] = (uint16_t)c;
                }
            }
    // per output row: window base row, then the V tap pairs padded to 8
    const int n = (int)hp.vbase.size();
    hp.vrow16.assign((size_t)n * 16, 0);
    for (int i = 0; i < n; ++i) {
        hp.vrow16[(size_t)i * 16] = hp.vbase[i];
        for (int j = 0; j < hp.vtp; ++j) hp.vrow16[(size_t)i * 16 + 1 + j] = hp.vcoef2[(size_t)i * hp.vtp + j];
    }
}

// strip_kernel packs an H row pair with v_cvt_pk_i16_i32, whose saturation
// stands in for hScale*To15's FFMIN(val >> sh, 32767): exact only if no output
// can fall below -32768 (the most negative sum: every negative tap on a
// full-scale sample).  Plans that could are left to scale_kernel.
bool strip_h_sat_ok(const HostPlane &hp, int depth) {
    const int64_t maxs = (1 << depth) - 1;
    const int sh = depth == 8 ? 7 : depth - 1;
    const int taps = hp.h.taps, n = (int)hp.h.pos.size();
    for (int x = 0; x < n; ++x) {
        int64_t neg = 0;
        for (int k = 0; k < taps; ++k) neg += std::min<int64_t>(0, hp.h.coef[(size_t)x * taps + k]);
        if ((neg * maxs) >> sh < -32768) return false;
    }
    return true;
}

inline int hw_bucket(int need) {
    static const int b[] = {3, 4, 5, 6, 8, 10, 12, 16};
    for (int v : b)
        if (need <= v) return v;
    return -1;
}

}  // namespace

#ifndef PIXPATH_DIRECT_CHO
#define PIXPATH_DIRECT_CHO 24
#endif
constexpr int kDirectCho = PIXPATH_DIRECT_CHO;  // strip_kernel DIRECT: tallest chunk (output rows)

// one_seg_chroma: chroma planes walk their whole height in one segment (the
// chain plan's second-stage vertical filter follows the first stage's rows)
static int plan_create(pp_ctx *ctx, int src_fmt, int sw, int sh, int dst_fmt, int dw, int dh, int flags, double p0,
                       double p1, bool one_seg_chroma, pp_scale_plan **out, int cho_max = 0, bool allow_direct = true) {
    using namespace pp;
    if (!out) PP_FAIL(PP_ERR_INVALID, "null argument");
    *out = nullptr;  // ctx == NULL: host-only plan (tables for introspection, no device upload)
    const bool force_generic = (flags & PP_PLAN_GENERIC) != 0;
    flags &= ~PP_PLAN_GENERIC;
    FmtInfo si = fmt_info(src_fmt), di = fmt_info(dst_fmt);
    if (!si.valid || si.packed) PP_FAIL(PP_ERR_INVALID, "source format %d must be planar YUV", src_fmt);
    if (!di.valid || dst_fmt == PP_FMT_V210) PP_FAIL(PP_ERR_INVALID, "destination format %d unsupported", dst_fmt);
    if (sw < 4 || sh < 4 || dw < 1 || dh < 1 || sw > 16384 || sh > 16384 || dw > 16384 || dh > 16384)
        PP_FAIL(PP_ERR_INVALID, "bad dimensions %dx%d -> %dx%d", sw, sh, dw, dh);
    if (!(flags & (PP_SWS_BICUBIC | PP_SWS_LANCZOS | PP_SWS_BILINEAR)))
        PP_FAIL(PP_ERR_UNSUPPORTED, "flags 0x%x: only bicubic, lanczos, bilinear", flags);

    std::unique_ptr<pp_scale_plan> P(new pp_scale_plan());
    P->ctx = ctx;
    P->src_fmt = src_fmt; P->dst_fmt = dst_fmt;
    P->sw = sw; P->sh = sh; P->dw = dw; P->dh = dh;
    P->si = si; P->di = di;
    P->csw = ceil_rshift(sw, si.hsub); P->csh = ceil_rshift(sh, si.vsub);
    P->cdw = ceil_rshift(dw, di.hsub); P->cdh = ceil_rshift(dh, di.vsub);

    // ff_get_unscaled_swscale(): converters tried before the generic path.
    if (sw == dw && sh == dh) {
        if (src_fmt == PP_FMT_YUV422P && dst_fmt == PP_FMT_UYVY422) {
            P->kind = pp_scale_plan::INTERLEAVE;
            *out = P.release();
            return PP_OK;
        }
        if (!di.packed && si.hsub == di.hsub && si.vsub == di.vsub && si.depth <= di.depth) {
            P->kind = pp_scale_plan::COPY;
            *out = P.release();
            return PP_OK;
        }
    }
    P->kind = di.packed ? pp_scale_plan::GENERIC_UYVY : pp_scale_plan::GENERIC;

    // sws_init_context(): increments and siting (get_local_pos, default -513)
    std::string err;
    const int lumXInc = (int)((((int64_t)sw << 16) + (dw >> 1)) / dw);
    const int lumYInc = (int)((((int64_t)sh << 16) + (dh >> 1)) / dh);
    const int chrXInc = (int)((((int64_t)P->csw << 16) + (P->cdw >> 1)) / P->cdw);
    const int chrYInc = (int)((((int64_t)P->csh << 16) + (P->cdh >> 1)) / P->cdh);
    if (P->f[0].build(lumXInc, sw, dw, 4, 1 << 14, flags, p0, p1, local_pos(0), local_pos(0), &err) ||
        P->f[1].build(chrXInc, P->csw, P->cdw, 4, 1 << 14, flags, p0, p1, local_pos(si.hsub), local_pos(di.hsub), &err) ||
        P->f[2].build(lumYInc, sh, dh, 2, 1 << 12, flags, p0, p1, local_pos(0), local_pos(0), &err) ||
        P->f[3].build(chrYInc, P->csh, P->cdh, 2, 1 << 12, flags, p0, p1, local_pos(si.vsub), local_pos(di.vsub), &err))
        PP_FAIL(PP_ERR_UNSUPPORTED, "filter construction: %s", err.c_str());

    // GPU layout: compact windows, one H-tap bucket for the launch
    HostPlane hp[2];
    for (int c = 0; c < 2; ++c) {
        const int src_w = c ? P->csw : sw, src_h = c ? P->csh : sh;
        if (P->f[c].compact(src_w, 1, &hp[c].h, &err) || P->f[2 + c].compact(src_h, 1, &hp[c].v, &err))
            PP_FAIL(PP_ERR_UNSUPPORTED, "%s", err.c_str());
    }
    const int ht = ht_bucket(std::max(hp[0].h.taps, hp[1].h.taps));
    if (ht < 0) PP_FAIL(PP_ERR_UNSUPPORTED, "horizontal filter of %d taps", std::max(hp[0].h.taps, hp[1].h.taps));
    P->ht = ht;
    for (int c = 0; c < 2; ++c) {
        const int src_w = c ? P->csw : sw, src_h = c ? P->csh : sh;
        const int dst_w = c ? P->cdw : dw, dst_h = c ? P->cdh : dh;
        if (hp[c].h.taps != ht && P->f[c].compact(src_w, ht, &hp[c].h, &err))
            PP_FAIL(PP_ERR_UNSUPPORTED, "%s", err.c_str());
        pair_rows(hp[c]);
        // chain plans (one_seg_chroma): the chroma ring of the fused second stage
        // needs the short chunks; PIXPATH_CHAIN_LUMA_CHO (measurement) sets luma's
        int cho_c = cho_max;
        if (!c && one_seg_chroma)
            if (const char *e = PP_KNOB("PIXPATH_CHAIN_LUMA_CHO")) cho_c = std::max(1, atoi(e));
        if (plan_tiles(hp[c], src_w, src_h, dst_w, dst_h, &P->lds_bytes, &err, c && one_seg_chroma ? 1 << 20 : 0, cho_c))
            PP_FAIL(PP_ERR_UNSUPPORTED, "%s", err.c_str());
    }
    // strip_kernel eligibility: the generic tiling fits 256-column strips,
    // <= 8 V tap pairs, one H window bucket for both planes, single-pass
    // staging, LDS within the budget.  Strip width 256; PIXPATH_STRIP_TW=512
    // (plain plans only, measurement) runs 512-column strips with 8 waves and
    // twice the LDS budget -- measured slower on every config (config 2
    // 1.554 vs 1.501 ms, config 3 10-bit 5.17 vs 4.87 ms, 8-bit 3.57 vs
    // 3.25 ms per 600-frame launch; profiles/r3/strip_tw_ab.txt).
    {
        const char *etw = PP_KNOB("PIXPATH_STRIP_TW");
        bool ok0 = !force_generic;
        const int CH = si.depth > 8 ? 8 : 16;
        for (int c = 0; c < 2 && ok0; ++c) ok0 = hp[c].tw == kTileW && hp[c].vtp <= 8 && strip_h_sat_ok(hp[c], si.depth);
        const int tw_first = (etw && atoi(etw) == 512 && !one_seg_chroma && !di.packed) ? 512 : 256;
        for (int ftw = tw_first; ok0 && ftw >= 256; ftw /= 2) {
            bool ok = true;
            int need = 1;
            for (int c = 0; c < 2 && ok; ++c) {
                fast_tiling(hp[c], c ? P->csw : sw, c ? P->cdw : dw, ftw);
                for (int v : hp[c].f_cn) ok = ok && (v + CH - 1) / CH <= ftw;
                if (!ok) break;
                fast_windows(hp[c], c ? P->cdw : dw);
                need = std::max(need, hp[c].hw_need);
            }
            const int HW = ok ? hw_bucket(need) : -1;
            size_t lds = 0;
            for (int c = 0; c < 2 && HW > 0; ++c) {
                fast_coefs(hp[c], c ? P->cdw : dw, HW);
                hp[c].S_fast = std::max(hp[c].f_S, (hp[c].max_base + 2 * HW + 15) & ~15);
                P->fast_lds_plane[c] = (size_t)hp[c].maxnew * hp[c].S_fast * 2 + (size_t)hp[c].ring * ftw * 2;
                lds = std::max(lds, P->fast_lds_plane[c]);
            }
            if (HW > 0 && lds <= lds_budget() * (size_t)(ftw / 256)) {
                P->fast_hw = HW;
                P->fast_lds = lds;
                P->fast_tw = ftw;
                break;
            }
        }
    }

    // strip_kernel DIRECT (8-bit sources, 8-dword windows, plain plans: the
    // 2:1 downscales of config 3): no staged rows, so the chunks are chosen
    // for the V window ring alone -- its own row tiling and chunk tables
    // (24-row chunks: 2.73 ms per 600-frame config-3 8-bit launch, against
    // 3.04 at the staged plan's 8 rows and 2.76 at 32, profiles/r5/)
    HostPlane hpd[2];
    if (P->fast_hw == 8 && si.depth == 8) {
        bool okd = allow_direct && !di.packed && !one_seg_chroma && P->fast_tw == 256;
        size_t dl = 0;
        for (int c = 0; c < 2 && okd; ++c) {
            hpd[c] = hp[c];
            size_t tmp = 0;
            okd = plan_tiles(hpd[c], c ? P->csw : sw, c ? P->csh : sh, c ? P->cdw : dw, c ? P->cdh : dh, &tmp, &err, 0,
                             kDirectCho, true) == 0 && hpd[c].tw == 256;
            dl = std::max(dl, (size_t)hpd[c].ring * 256 * 2);
        }
        if (okd) {
            P->direct = true;
            P->fast_lds = dl;
        }
    }

    // launch geometry of every plane (host-only plans too: introspection, chain planning)
    {
        int base = 0;
        for (int p = 0; p < 3; ++p) {
            const int c = p ? 1 : 0;
            PlaneJob &J = P->job[p];
            J.sw = c ? P->csw : sw; J.sh = c ? P->csh : sh;
            J.dw = c ? P->cdw : dw; J.dh = c ? P->cdh : dh;
            J.tiles_x = hp[c].tiles_x; J.tiles_y = hp[c].nseg; J.tw = hp[c].tw;
            J.twl = 0;
            while ((1 << J.twl) < J.tw) ++J.twl;
            J.seg_h = hp[c].seg_h; J.cho = hp[c].cho;
            J.tile_base = base;
            base += J.tiles_x * J.tiles_y;
            J.vtp = hp[c].vtp; J.ring = hp[c].ring; J.maxnew = hp[c].maxnew; J.S = hp[c].S;
            J.dither_off = p == 2 ? 3 : 0;
        }
        int fbase = 0;
        for (int p = 0; p < 3; ++p) {  // strip_kernel jobs: its own strip width
            const int c = p ? 1 : 0;
            PlaneJob &F = P->fjob[p];
            F = P->job[p];
            F.S = hp[c].S_fast;
            if (P->fast_hw) {
                F.tiles_x = hp[c].f_tiles_x;
                F.tw = P->fast_tw;
                F.twl = P->fast_tw == 512 ? 9 : 8;
            }
            if (P->direct) {
                F.tiles_y = hpd[c].nseg; F.seg_h = hpd[c].seg_h; F.cho = hpd[c].cho;
                F.ring = hpd[c].ring; F.maxnew = 0;
            }
            F.tile_base = fbase;
            fbase += F.tiles_x * F.tiles_y;
        }
        P->fast_tiles = fbase;
    }
    if (one_seg_chroma) {  // the chain plan re-sizes the chroma staging for its segments
        P->chroma_lo = hp[1].lo;
        P->chroma_hi = hp[1].hi;
    }
    if (!ctx) {
        *out = P.release();
        return PP_OK;
    }
    // one device allocation for every table
    auto sz4 = [](size_t n) { return (n * 4 + 255) & ~size_t(255); };
    auto sz2 = [](size_t n) { return (n * 2 + 255) & ~size_t(255); };
    size_t total = 0;
    for (int c = 0; c < 2; ++c)
        total += sz4(hp[c].h.pos.size()) + sz2(hp[c].h.coef.size()) + sz4(hp[c].vbase.size()) +
                 sz4(hp[c].vcoef2.size()) + 2 * sz4(hp[c].c0.size()) + 2 * sz4(hp[c].lo.size()) +
                 sz4(hp[c].hbase4.size()) + sz4(hp[c].hcoefw.size()) + sz4(hp[c].vrow16.size()) +
                 sz4(hp[c].f_c0.size()) + sz4(hp[c].f_cn.size()) + 2 * sz4(hpd[c].lo.size());
    PP_HIP(hipSetDevice(ctx->device));
    PP_HIP(hipMalloc(&P->dev, total));
    std::vector<uint8_t> host(total, 0);
    size_t off = 0;
    const int32_t *dptr32[2][14] = {};
    const int16_t *dptr16[2][1];
    auto put = [&](const void *src, size_t bytes, size_t padded) {
        std::memcpy(host.data() + off, src, bytes);
        const void *d = static_cast<uint8_t *>(P->dev) + off;
        off += padded;
        return d;
    };
    for (int c = 0; c < 2; ++c) {
        dptr32[c][0] = (const int32_t *)put(hp[c].h.pos.data(), hp[c].h.pos.size() * 4, sz4(hp[c].h.pos.size()));
        dptr16[c][0] = (const int16_t *)put(hp[c].h.coef.data(), hp[c].h.coef.size() * 2, sz2(hp[c].h.coef.size()));
        dptr32[c][1] = (const int32_t *)put(hp[c].vbase.data(), hp[c].vbase.size() * 4, sz4(hp[c].vbase.size()));
        dptr32[c][6] = (const int32_t *)put(hp[c].vcoef2.data(), hp[c].vcoef2.size() * 4, sz4(hp[c].vcoef2.size()));
        dptr32[c][2] = (const int32_t *)put(hp[c].c0.data(), hp[c].c0.size() * 4, sz4(hp[c].c0.size()));
        dptr32[c][3] = (const int32_t *)put(hp[c].cn.data(), hp[c].cn.size() * 4, sz4(hp[c].cn.size()));
        dptr32[c][4] = (const int32_t *)put(hp[c].lo.data(), hp[c].lo.size() * 4, sz4(hp[c].lo.size()));
        dptr32[c][5] = (const int32_t *)put(hp[c].hi.data(), hp[c].hi.size() * 4, sz4(hp[c].hi.size()));
        if (P->fast_hw) {
            dptr32[c][7] = (const int32_t *)put(hp[c].hbase4.data(), hp[c].hbase4.size() * 4, sz4(hp[c].hbase4.size()));
            dptr32[c][8] = (const int32_t *)put(hp[c].hcoefw.data(), hp[c].hcoefw.size() * 4, sz4(hp[c].hcoefw.size()));
            dptr32[c][9] = (const int32_t *)put(hp[c].vrow16.data(), hp[c].vrow16.size() * 4, sz4(hp[c].vrow16.size()));
            dptr32[c][10] = (const int32_t *)put(hp[c].f_c0.data(), hp[c].f_c0.size() * 4, sz4(hp[c].f_c0.size()));
            dptr32[c][11] = (const int32_t *)put(hp[c].f_cn.data(), hp[c].f_cn.size() * 4, sz4(hp[c].f_cn.size()));
        }
        if (P->direct) {
            dptr32[c][12] = (const int32_t *)put(hpd[c].lo.data(), hpd[c].lo.size() * 4, sz4(hpd[c].lo.size()));
            dptr32[c][13] = (const int32_t *)put(hpd[c].hi.data(), hpd[c].hi.size() * 4, sz4(hpd[c].hi.size()));
        }
    }
    PP_HIP(hipMemcpy(P->dev, host.data(), total, hipMemcpyHostToDevice));

    for (int p = 0; p < 3; ++p) {
        const int c = p ? 1 : 0;
        PlaneJob &J = P->job[p];
        J.hpos = dptr32[c][0]; J.hcoef = dptr16[c][0];
        J.vbase = dptr32[c][1]; J.vcoef2 = dptr32[c][6];
        J.tile_c0 = dptr32[c][2]; J.tile_cn = dptr32[c][3];
        J.chunk_lo = dptr32[c][4]; J.chunk_hi = dptr32[c][5];
        J.hbase4 = dptr32[c][7]; J.hcoefw = dptr32[c][8]; J.vrow16 = dptr32[c][9];
        PlaneJob &F = P->fjob[p];
        F.hpos = J.hpos; F.hcoef = J.hcoef; F.vbase = J.vbase; F.vcoef2 = J.vcoef2;
        F.chunk_lo = J.chunk_lo; F.chunk_hi = J.chunk_hi;
        F.hbase4 = J.hbase4; F.hcoefw = J.hcoefw; F.vrow16 = J.vrow16;
        F.tile_c0 = P->fast_hw ? dptr32[c][10] : J.tile_c0;
        F.tile_cn = P->fast_hw ? dptr32[c][11] : J.tile_cn;
        if (P->direct) {
            F.chunk_lo = dptr32[c][12];
            F.chunk_hi = dptr32[c][13];
        }
    }
    *out = P.release();
    return PP_OK;
}

extern "C" int pp_scale_plan_create(pp_ctx *ctx, int src_fmt, int sw, int sh, int dst_fmt, int dw, int dh,
                                    int flags, double p0, double p1, pp_scale_plan **out) {
    return plan_create(ctx, src_fmt, sw, sh, dst_fmt, dw, dh, flags, p0, p1, false, out);
}

namespace {

// An FFmpeg "unscaled" filter bank (initFilter's |xInc - 0x10000| < 10 case):
// output i takes input i with the single tap `one`.
bool identity_bank(const pp::FilterBank &f, int one) {
    for (int i = 0; i < f.n; ++i)
        for (int j = 0; j < f.size; ++j) {
            const int16_t c = f.coef[(size_t)i * f.size + j];
            if (f.pos[i] + j == i ? c != one : c != 0) return false;
        }
    return true;
}

}  // namespace

#ifndef PIXPATH_CHAIN_CHO
#define PIXPATH_CHAIN_CHO 16
#endif
constexpr int kChainCho = PIXPATH_CHAIN_CHO;
#ifndef PIXPATH_CHAIN_SEG2
#define PIXPATH_CHAIN_SEG2 4
#endif
constexpr int kChainSeg2 = PIXPATH_CHAIN_SEG2;  // second-stage segments of a chain plan's chroma planes

// create_avpvs_segment's two stages (lib/ffmpeg.py:1037-1048): the scale
// filter writes the overlay's yuv420p (overlay's default format=yuv420), then
// libavfilter converts yuv420p -> dst_fmt at the same size with a second
// swscale context (bicubic).  Both stages in one strip_kernel launch when the
// first stage is a strip plan and the second stage's luma / horizontal chroma
// filters are FFmpeg's identity banks (always, for the AVPVS formats).
extern "C" int pp_scale_chain_plan_create(pp_ctx *ctx, int src_fmt, int sw, int sh, int dst_fmt, int dw, int dh,
                                          int flags, double p0, double p1, pp_scale_plan **out) {
    using namespace pp;
    if (!out) PP_FAIL(PP_ERR_INVALID, "null argument");
    *out = nullptr;
    if (dst_fmt != PP_FMT_YUV420P && dst_fmt != PP_FMT_YUV422P && dst_fmt != PP_FMT_YUV420P10LE &&
        dst_fmt != PP_FMT_YUV422P10LE)
        PP_FAIL(PP_ERR_INVALID, "chain target %d: yuv420p, yuv422p, yuv420p10le or yuv422p10le", dst_fmt);
    if (dst_fmt == PP_FMT_YUV420P)  // no conversion after the overlay
        return plan_create(ctx, src_fmt, sw, sh, dst_fmt, dw, dh, flags, p0, p1, false, out);
    pp_scale_plan *s1 = nullptr, *p2 = nullptr;
    // 16-row chunks: the LDS ring of the second stage then still leaves 6
    // workgroups per CU (32-row chunks: 2.73 vs 2.30 ms per 600-frame config-4
    // canvas launch, profiles/r2/chain_ab.log)
    int rc = plan_create(ctx, src_fmt, sw, sh, PP_FMT_YUV420P, dw, dh, flags, p0, p1, true, &s1, kChainCho, false);
    if (rc) return rc;
    std::unique_ptr<pp_scale_plan> P(s1);
    rc = plan_create(ctx, PP_FMT_YUV420P, dw, dh, dst_fmt, dw, dh, PP_SWS_BICUBIC, PP_SWS_PARAM_DEFAULT,
                     PP_SWS_PARAM_DEFAULT, false, &p2);
    if (rc) return rc;
    P->first_kind = P->kind;
    P->kind = pp_scale_plan::CHAIN;
    P->stage2 = p2;
    const FmtInfo di = fmt_info(dst_fmt);
    P->chain_out = di.depth;
    P->dst_fmt = dst_fmt;
    if ((p2->kind != pp_scale_plan::GENERIC && p2->kind != pp_scale_plan::COPY) || !P->fast_hw) {
        *out = P.release();
        return PP_OK;
    }
    const bool v422 = di.vsub == 0;
    // COPY (yuv420p -> yuv420p10le, planarCopyWrapper) is x << 2 as well
    bool ok = p2->kind == pp_scale_plan::COPY ||
              (identity_bank(p2->f[0], 1 << 14) && identity_bank(p2->f[1], 1 << 14) &&
               identity_bank(p2->f[2], 1 << 12) && (v422 || identity_bank(p2->f[3], 1 << 12)));
    std::vector<int32_t> vrow2, chunk2, seg2;
    int vtp2 = 0, ring2 = 0, maxnew2 = 0;
    if (ok && v422) {
        // second-stage chroma rows: compact window, tap pairs, record per row
        const int cdh1 = P->cdh, dh2 = p2->cdh;
        HostPlane h2;
        std::string err;
        if (p2->f[3].compact(cdh1, 1, &h2.v, &err)) PP_FAIL(PP_ERR_UNSUPPORTED, "%s", err.c_str());
        std::vector<int> need(dh2, 0);
        for (int r = 0; r < dh2; ++r) {
            int last = 0;
            for (int k = 0; k < h2.v.taps; ++k)
                if (h2.v.coef[(size_t)r * h2.v.taps + k]) last = k;
            need[r] = h2.v.pos[r] + last;
        }
        // rows in pairs (2m, 2m + 1) over one shared window (strip.hpp pass2):
        // base = the even row at or below the pair's first non-zero tap, each
        // row's non-zero taps placed at their rows within the window
        const int npair = (dh2 + 1) / 2, T2 = h2.v.taps;
        auto tap_rows = [&](int r, int *lo, int *hi) {
            *lo = INT32_MAX;
            *hi = -1;
            for (int k = 0; k < T2; ++k)
                if (h2.v.coef[(size_t)r * T2 + k]) {
                    *lo = std::min(*lo, h2.v.pos[r] + k);
                    *hi = std::max(*hi, h2.v.pos[r] + k);
                }
            if (*hi < 0) *lo = *hi = h2.v.pos[r];  // an all-zero row (none in practice)
        };
        std::vector<int> pbase(npair);
        vtp2 = 1;
        for (int m = 0; m < npair; ++m) {
            int la, ha, lb, hb;
            tap_rows(2 * m, &la, &ha);
            tap_rows(std::min(2 * m + 1, dh2 - 1), &lb, &hb);
            pbase[m] = std::min(la, lb) & ~1;
            vtp2 = std::max(vtp2, (std::max(ha, hb) - pbase[m]) / 2 + 1);
        }
        ok = vtp2 <= 3;  // strip.hpp pass2 instances (registers: spill-free at 6 waves)
        vrow2.assign((size_t)npair * 16, 0);
        for (int m = 0; ok && m < npair; ++m) {
            vrow2[(size_t)m * 16] = pbase[m];
            uint16_t *t16 = reinterpret_cast<uint16_t *>(&vrow2[(size_t)m * 16 + 1]);
            for (int h = 0; h < 2 && 2 * m + h < dh2; ++h)
                for (int k = 0; k < T2; ++k) {
                    const int16_t c = h2.v.coef[(size_t)(2 * m + h) * T2 + k];
                    if (!c) continue;
                    const int y = h2.v.pos[2 * m + h] + k - pbase[m];  // in [0, 2 * vtp2)
                    t16[2 * (h * vtp2 + y / 2) + (y & 1)] = (uint16_t)c;
                }
        }
        // per first-stage chunk: the second-stage rows it completes and the ring2 rows kept
        const int cho = P->fjob[1].cho, nch = (cdh1 + cho - 1) / cho;
        chunk2.assign((size_t)nch * 4, 0);
        int done = 0;
        for (int ci = 0; ci < nch; ++ci) {
            const int y0 = ci * cho, end = std::min(cdh1, y0 + cho);
            const int lo2 = done;
            // pairs complete together (a pair's rows are computed at once)
            while (done < dh2 && need[done] < end && (done + 1 >= dh2 || need[done + 1] < end))
                done = std::min(dh2, done + 2);
            if (ci == nch - 1) done = dh2;
            const int b2 = (std::min(lo2 < dh2 ? pbase[lo2 / 2] : y0, y0)) & ~1;
            chunk2[4 * ci] = lo2;
            chunk2[4 * ci + 1] = done;
            chunk2[4 * ci + 2] = b2;
            chunk2[4 * ci + 3] = (y0 - b2 + 1) >> 1;
            int top = end;
            for (int m = lo2 / 2; m < (done + 1) / 2; ++m) top = std::max(top, pbase[m] + 2 * vtp2);
            ring2 = std::max(ring2, top - b2);
        }
        ring2 = (ring2 + 1) & ~1;
        // segments of the second-stage rows (the first stage's chroma walk is
        // one segment so that the second stage's taps are always in ring2):
        // each segment's walk starts at the chunk of its first row's window
        // and ends at the chunk that completes its last row, recomputing the
        // few first-stage rows of the halo instead of one 1080-row workgroup
        // per strip (4,800 long workgroups per 600-frame launch: a tail)
        int nseg2 = kChainSeg2;
        if (const char *e = PP_KNOB("PIXPATH_CHAIN_SEG2")) nseg2 = std::max(1, atoi(e));
        nseg2 = std::min(nseg2, std::max(1, dh2 / 16));
        seg2.assign((size_t)nseg2 * 4, 0);
        for (int sg = 0; sg < nseg2; ++sg) {
            // segments start on a row pair
            const int r0 = (int)((int64_t)sg * dh2 / nseg2) & ~1;
            const int r1 = sg + 1 == nseg2 ? dh2 : (int)((int64_t)(sg + 1) * dh2 / nseg2) & ~1;
            seg2[4 * sg] = pbase[r0 / 2] / cho * cho;
            seg2[4 * sg + 1] = std::min(cdh1, (need[r1 - 1] / cho + 1) * cho);
            seg2[4 * sg + 2] = r0;
            seg2[4 * sg + 3] = r1;
            // a segment's first chunk stages its whole source window, not only
            // the rows new to a walk from the top: the staging buffer grows to it
            const int c0 = seg2[4 * sg] / cho;
            maxnew2 = std::max(maxnew2, P->chroma_hi[c0] - P->chroma_lo[c0]);
        }
    }
    if (maxnew2 > P->fjob[1].maxnew) {
        for (int p = 1; p < 3; ++p) P->fjob[p].maxnew = maxnew2;
        P->fast_lds_plane[1] = (size_t)maxnew2 * P->fjob[1].S * 2 + (size_t)P->fjob[1].ring * P->fast_tw * 2;
        P->fast_lds = std::max(P->fast_lds, P->fast_lds_plane[1]);
    }
    // the byte ring is circular: a power of two of rows >= every chunk's live span
    int r2rows = 2;
    while (r2rows < ring2) r2rows <<= 1;
    const size_t lds = P->fast_lds + (ring2 ? (size_t)r2rows * P->fast_tw : 0);
    if (!ok || lds > 64 * 1024) {
        *out = P.release();
        return PP_OK;
    }
    // luma as its own launch (4:2:2 targets: the chroma launch then carries
    // only the ring2 planes): its plan is the plain first stage, same filters
    pp_scale_plan *lp = nullptr;
    // PIXPATH_CHAIN_ONE_LAUNCH (measurement build): keep luma in the chroma launch
    if (v422 && !PP_KNOB("PIXPATH_CHAIN_ONE_LAUNCH") &&
        plan_create(ctx, src_fmt, sw, sh, PP_FMT_YUV420P, dw, dh, flags, p0, p1, false, &lp,
                    PP_KNOB("PIXPATH_CHAIN_LUMA_CHO") ? std::atoi(PP_KNOB("PIXPATH_CHAIN_LUMA_CHO")) : 0, false) == PP_OK) {
        if (lp->kind == pp_scale_plan::GENERIC && lp->fast_hw > 0 && lp->fast_tw == 256) {
            P->luma = lp;
            lp->fjob[0].fuse = P->chain_out > 8 ? 1 : 0;
        } else {
            (void)pp_scale_plan_destroy(lp);
        }
    }
    const size_t chain_lds = P->luma ? P->fast_lds_plane[1] + (size_t)r2rows * P->fast_tw : lds;
    if (!ctx) {  // host-only plan: introspection (pp_scale_plan_path / _stats) only
        P->chain_fused = true;
        P->chain_lds = chain_lds;
        *out = P.release();
        return PP_OK;
    }
    const size_t b1 = (vrow2.size() * 4 + 255) & ~size_t(255), b2 = (chunk2.size() * 4 + 255) & ~size_t(255);
    if (v422) {
        PP_HIP(hipMalloc(&P->dev2, b1 + b2 + seg2.size() * 4));
        PP_HIP(hipMemcpy(P->dev2, vrow2.data(), vrow2.size() * 4, hipMemcpyHostToDevice));
        PP_HIP(hipMemcpy(static_cast<uint8_t *>(P->dev2) + b1, chunk2.data(), chunk2.size() * 4, hipMemcpyHostToDevice));
        PP_HIP(hipMemcpy(static_cast<uint8_t *>(P->dev2) + b1 + b2, seg2.data(), seg2.size() * 4, hipMemcpyHostToDevice));
    }
    const int widen = P->chain_out > 8 ? 1 : 0;
    for (int p = 0; p < 3; ++p) {
        PlaneJob &J = P->fjob[p];
        J.fuse = (p && v422) ? 2 : widen;
        if (J.fuse == 2) {
            J.vtp2 = vtp2;
            J.r2mask = r2rows - 1;
            J.vrow2 = static_cast<const int32_t *>(P->dev2);
            J.chunk2 = reinterpret_cast<const int32_t *>(static_cast<uint8_t *>(P->dev2) + b1);
            J.seg2 = reinterpret_cast<const int32_t *>(static_cast<uint8_t *>(P->dev2) + b1 + b2);
            J.tiles_y = (int)seg2.size() / 4;
        }
    }
    P->chain_fused = true;
    P->chain_lds = chain_lds;
    *out = P.release();
    return PP_OK;
}

extern "C" int pp_scale_plan_destroy(pp_scale_plan *P) {
    if (!P) return PP_OK;
    if (P->stage2) (void)pp_scale_plan_destroy(P->stage2);
    if (P->luma) (void)pp_scale_plan_destroy(P->luma);
    if (P->side) (void)hipStreamDestroy(P->side);
    if (P->fork) (void)hipEventDestroy(P->fork);
    if (P->join) (void)hipEventDestroy(P->join);
    if (P->dev2) (void)hipFree(P->dev2);
    if (P->dev) (void)hipFree(P->dev);
    if (P->scratch) (void)hipFree(P->scratch);
    delete P;
    return PP_OK;
}

extern "C" int pp_scale_plan_path(const pp_scale_plan *P) {
    if (!P) PP_FAIL(PP_ERR_INVALID, "null plan");
    if (P->kind == pp_scale_plan::CHAIN) return P->chain_fused ? P->fast_hw : 0;
    return (P->kind == pp_scale_plan::GENERIC || P->kind == pp_scale_plan::GENERIC_UYVY) ? P->fast_hw : 0;
}

extern "C" int pp_scale_plan_stats(const pp_scale_plan *P, int64_t *out, int n) {
    if (!P || !out || n < 0) PP_FAIL(PP_ERR_INVALID, "null argument");
    if (P->kind == pp_scale_plan::COPY || P->kind == pp_scale_plan::INTERLEAVE) return 0;
    const bool strip = P->fast_hw > 0;
    const pp::PlaneJob &L = strip ? P->fjob[0] : P->job[0];
    const bool chain = P->kind == pp_scale_plan::CHAIN && P->chain_fused;
    const int64_t v[] = {(int64_t)(chain ? P->chain_lds : strip ? P->fast_lds : P->lds_bytes),
                         strip ? P->fast_tw : pp::kThreads,
                         strip ? P->fast_tiles : P->job[2].tile_base + P->job[2].tiles_x * P->job[2].tiles_y, L.cho,
                         L.seg_h, L.vtp,
                         P->job[1].vtp, L.S, L.ring, L.maxnew};
    const int k = std::min<int>(n, (int)(sizeof(v) / sizeof(v[0])));
    for (int i = 0; i < k; ++i) out[i] = v[i];
    return k;
}

extern "C" int pp_scale_plan_filter(const pp_scale_plan *P, int which, int16_t *coef, int32_t *pos, int capacity) {
    if (!P || which < 0 || which > 3) PP_FAIL(PP_ERR_INVALID, "bad plan/which");
    if (P->kind == pp_scale_plan::COPY || P->kind == pp_scale_plan::INTERLEAVE) return 0;
    const pp::FilterBank &f = P->f[which];
    if ((int64_t)f.n * f.size > capacity) PP_FAIL(PP_ERR_INVALID, "capacity %d < %d", capacity, f.n * f.size);
    std::memcpy(coef, f.coef.data(), f.coef.size() * 2);
    std::memcpy(pos, f.pos.data(), f.pos.size() * 4);
    return f.size;
}

namespace {

bool aligned(const void *p, int64_t ls, int64_t fs, int a) {
    return ((uintptr_t)p % a) == 0 && ls % a == 0 && fs % a == 0;
}

int launch_generic(pp_scale_plan *P, const pp_frames *src, const pp_frames *dst, int nframes, hipStream_t st,
                   int out_depth, bool allow_dither) {
    using namespace pp;
    ScaleArgs a{};
    a.nplanes = 3;
    for (int p = 0; p < 3; ++p) {
        a.pl[p] = P->job[p];
        a.src[p] = static_cast<const uint8_t *>(src->data[p]);
        a.sls[p] = src->linesize[p];
        a.sfs[p] = src->frame_stride[p];
        a.dst[p] = static_cast<uint8_t *>(dst->data[p]);
        a.dls[p] = dst->linesize[p];
        a.dfs[p] = dst->frame_stride[p];
    }
    a.hshift = P->si.depth == 8 ? 7 : P->si.depth - 1;
    a.dither = allow_dither && P->si.depth > 8 && out_depth == 8;
    a.vec_src = 1;
    a.vec_dst = 1;
    if (const char *e = PP_KNOB("PIXPATH_SCALE_DEBUG")) a.debug = atoi(e);
    for (int p = 0; p < 3; ++p) {
        a.vec_src &= aligned(a.src[p], a.sls[p], nframes > 1 ? a.sfs[p] : 0, 16);
        a.vec_dst &= aligned(a.dst[p], a.dls[p], nframes > 1 ? a.dfs[p] : 0, out_depth == 8 ? 4 : 8);
    }
    const bool tw256 = P->job[0].tw == kTileW && P->job[1].tw == kTileW && P->job[2].tw == kTileW;
    KernelFn k;
    size_t lds = P->lds_bytes;
    int tiles = P->job[2].tile_base + P->job[2].tiles_x * P->job[2].tiles_y, threads = kThreads;
    // (an 8-bit HW-8 plan takes the strip path only with its DIRECT tiling:
    // that instance stages no rows)
    if (P->fast_hw && a.vec_src && (P->direct || !(P->si.depth == 8 && P->fast_hw == 8))) {
        for (int p = 0; p < 3; ++p) a.pl[p] = P->fjob[p];
        lds = P->fast_lds;
        tiles = P->fast_tiles;
        threads = P->fast_tw;
        const int vtm = strip_vtm_bucket(std::max(P->fjob[0].vtp, P->fjob[1].vtp));
        k = P->si.depth == 8 ? pick_strip_u8(out_depth, P->fast_hw, vtm, P->fast_tw)
                             : pick_strip_u16(out_depth, P->fast_hw, vtm, P->fast_tw);

    } else if (P->si.depth == 8) {
        k = out_depth == 8 ? pick_ht<uint8_t, 8>(P->ht, tw256) : pick_ht<uint8_t, 10>(P->ht, tw256);
    } else {
        k = out_depth == 8 ? pick_ht<uint16_t, 8>(P->ht, tw256) : pick_ht<uint16_t, 10>(P->ht, tw256);
    }
    if (!k) PP_FAIL(PP_ERR_UNSUPPORTED, "no kernel for %d taps", P->ht);
    a.tiles = tiles;
    const int fmax = std::max(1, (1 << 30) / tiles);  // 1-D grid size limit
    for (int f0 = 0; f0 < nframes; f0 += fmax) {
        const int nf = std::min(fmax, nframes - f0);
        ScaleArgs b = a;
        for (int p = 0; p < 3; ++p) {
            b.src[p] += f0 * a.sfs[p];
            b.dst[p] += f0 * a.dfs[p];
        }
        hipLaunchKernelGGL(k, dim3(tiles * nf), dim3(threads), lds, st, b);
    }
    PP_HIP(hipGetLastError());
    return PP_OK;
}

// GENERIC_UYVY on the strip path: one strip_kernel<.., FUSE = 1> launch whose
// planes store straight into the uyvy422 rows (U Y V Y byte order)
int launch_packed(pp_scale_plan *P, const pp_frames *src, const pp_frames *dst, int nframes, hipStream_t st) {
    using namespace pp;
    ScaleArgs a{};
    a.nplanes = 3;
    static const int off[3] = {1, 0, 2}, step[3] = {2, 4, 4};
    for (int p = 0; p < 3; ++p) {
        a.pl[p] = P->fjob[p];
        a.pl[p].pk_off = off[p];
        a.pl[p].pk_step = step[p];
        a.src[p] = static_cast<const uint8_t *>(src->data[p]);
        a.sls[p] = src->linesize[p];
        a.sfs[p] = src->frame_stride[p];
        a.dst[p] = static_cast<uint8_t *>(dst->data[0]);
        a.dls[p] = dst->linesize[0];
        a.dfs[p] = dst->frame_stride[0];
    }
    a.hshift = P->si.depth == 8 ? 7 : P->si.depth - 1;
    a.dither = 0;  // yuv2packedX rounds with 1 << 18, never dithers
    a.vec_src = 1;
    a.vec_dst = 0;
    const int vtm = strip_vtm_bucket(std::max(P->fjob[0].vtp, P->fjob[1].vtp));
    KernelFn k = P->si.depth == 8 ? pick_strip_packed_u8(P->fast_hw, vtm) : pick_strip_packed_u16(P->fast_hw, vtm);
    if (!k) PP_FAIL(PP_ERR_UNSUPPORTED, "no packed kernel for window %d", P->fast_hw);
    const int tiles = P->fast_tiles;
    a.tiles = tiles;
    const int fmax = std::max(1, (1 << 30) / tiles);
    for (int f0 = 0; f0 < nframes; f0 += fmax) {
        const int nf = std::min(fmax, nframes - f0);
        ScaleArgs b = a;
        for (int p = 0; p < 3; ++p) {
            b.src[p] += f0 * a.sfs[p];
            b.dst[p] += f0 * a.dfs[p];
        }
        hipLaunchKernelGGL(k, dim3(tiles * nf), dim3(kThreads), P->fast_lds, st, b);
    }
    PP_HIP(hipGetLastError());
    return PP_OK;
}

// CHAIN, fused: strip_kernel<.., FUSE = target depth> launches over the
// planes `pl` (job, source / destination plane index), tile bases renumbered
// for the launch
int launch_chain_planes(pp_scale_plan *P, const pp::PlaneJob *const *jobs, const int *pl, int np, int hw, size_t lds,
                        const pp_frames *src, const pp_frames *dst, int nframes, hipStream_t st,
                        bool luma_only = false) {
    using namespace pp;
    ScaleArgs a{};
    a.nplanes = np;
    int tiles = 0, vtp = 1;
    for (int i = 0; i < np; ++i) {
        const int p = pl[i];
        a.pl[i] = *jobs[i];
        a.pl[i].tile_base = tiles;
        tiles += a.pl[i].tiles_x * a.pl[i].tiles_y;
        vtp = std::max(vtp, a.pl[i].vtp);
        a.src[i] = static_cast<const uint8_t *>(src->data[p]);
        a.sls[i] = src->linesize[p];
        a.sfs[i] = src->frame_stride[p];
        a.dst[i] = static_cast<uint8_t *>(dst->data[p]);
        a.dls[i] = dst->linesize[p];
        a.dfs[i] = dst->frame_stride[p];
    }
    a.hshift = P->si.depth == 8 ? 7 : P->si.depth - 1;
    a.dither = P->si.depth > 8;
    a.vec_src = 1;
    a.vec_dst = 1;
    if (const char *e = PP_KNOB("PIXPATH_SCALE_DEBUG")) a.debug = atoi(e);
    for (int i = 0; i < np; ++i)
        a.vec_dst &= aligned(a.dst[i], a.dls[i], nframes > 1 ? a.dfs[i] : 0, P->chain_out == 8 ? 4 : 8);
    const int vtm = strip_vtm_bucket(vtp);
    // the luma launch of a 10-bit chain (fuse 1 into 10 bits) takes its own
    // instance without the ring2 / second-stage code (FUSE 9)
    // (clamped plans only: every plane's width a multiple of 4 with vector
    // stores, so those instances compile the clamped V pass alone)
    bool clamped = a.vec_dst != 0;
    for (int i = 0; i < np; ++i) clamped = clamped && (jobs[i]->dw & 3) == 0;
    const bool l9 = clamped && luma_only && P->chain_out == 10 && jobs[0]->fuse == 1 && !PP_KNOB("PIXPATH_CHAIN_NO_LUMA9");
    // ... and the chroma launch (every plane fuse 2) FUSE 11
    bool c11 = clamped && !luma_only && P->luma && P->chain_out == 10 && !PP_KNOB("PIXPATH_CHAIN_NO_CHROMA11");
    for (int i = 0; i < np; ++i) c11 = c11 && jobs[i]->fuse == 2;
    const bool u8 = P->si.depth == 8;
    KernelFn k = l9 ? (u8 ? pick_strip_luma_u8(hw, vtm) : pick_strip_luma_u16(hw, vtm))
                    : c11 ? (u8 ? pick_strip_chroma_u8(hw, vtm) : pick_strip_chroma_u16(hw, vtm)) : nullptr;
    if (!k)  // (FUSE 9 / 11 exist for narrow windows only)
        k = u8 ? pick_strip_chain_u8(P->chain_out, hw, vtm) : pick_strip_chain_u16(P->chain_out, hw, vtm);
    if (!k) PP_FAIL(PP_ERR_UNSUPPORTED, "no chain kernel for window %d", hw);
    a.tiles = tiles;
    const int fmax = std::max(1, (1 << 30) / tiles);
    for (int f0 = 0; f0 < nframes; f0 += fmax) {
        const int nf = std::min(fmax, nframes - f0);
        ScaleArgs b = a;
        for (int i = 0; i < np; ++i) {
            b.src[i] += f0 * a.sfs[i];
            b.dst[i] += f0 * a.dfs[i];
        }
        hipLaunchKernelGGL(k, dim3(tiles * nf), dim3(kThreads), lds, st, b);
    }
    PP_HIP(hipGetLastError());
    return PP_OK;
}

// CHAIN, fused: one launch over all planes, or (P->luma) the luma launch of
// the plain first-stage plan, then the chroma planes' chain launch
int launch_chain(pp_scale_plan *P, const pp_frames *src, const pp_frames *dst, int nframes, hipStream_t st) {
    using namespace pp;
    if (P->luma && P->luma->fast_hw == P->fast_hw && PP_KNOB("PIXPATH_CHAIN_COMBINED")) {
        // measurement: the luma plan's job (32-row chunks) and the chroma
        // chain jobs in ONE launch, LDS the larger of the two layouts
        const PlaneJob *jobs[3] = {&P->luma->fjob[0], &P->fjob[1], &P->fjob[2]};
        const int pl[3] = {0, 1, 2};
        return launch_chain_planes(P, jobs, pl, 3, P->fast_hw, std::max(P->luma->fast_lds_plane[0], P->chain_lds), src,
                                   dst, nframes, st);
    }
    if (P->luma) {
        // PIXPATH_CHAIN_OVERLAP (measurement build): the luma launch on a side
        // stream, concurrent with the chroma launch (fork / join events on `st`)
        const bool overlap = PP_KNOB("PIXPATH_CHAIN_OVERLAP") != nullptr;
        hipStream_t ls = st;
        if (overlap) {
            if (!P->side) {
                PP_HIP(hipStreamCreateWithFlags(&P->side, hipStreamNonBlocking));
                PP_HIP(hipEventCreateWithFlags(&P->fork, hipEventDisableTiming));
                PP_HIP(hipEventCreateWithFlags(&P->join, hipEventDisableTiming));
            }
            PP_HIP(hipEventRecord(P->fork, st));
            PP_HIP(hipStreamWaitEvent(P->side, P->fork, 0));
            ls = P->side;
        }
        const PlaneJob *lj[1] = {&P->luma->fjob[0]};
        const int lpl[1] = {0};
        if (int rc = launch_chain_planes(P, lj, lpl, 1, P->luma->fast_hw, P->luma->fast_lds_plane[0], src, dst,
                                         nframes, ls, true))
            return rc;
        const PlaneJob *cj[2] = {&P->fjob[1], &P->fjob[2]};
        const int cpl[2] = {1, 2};
        const int rc = launch_chain_planes(P, cj, cpl, 2, P->fast_hw, P->chain_lds, src, dst, nframes, st);
        if (overlap) {
            PP_HIP(hipEventRecord(P->join, P->side));
            PP_HIP(hipStreamWaitEvent(st, P->join, 0));
        }
        return rc;
    }
    const PlaneJob *jobs[3] = {&P->fjob[0], &P->fjob[1], &P->fjob[2]};
    const int pl[3] = {0, 1, 2};
    return launch_chain_planes(P, jobs, pl, 3, P->fast_hw, P->chain_lds, src, dst, nframes, st);
}

}  // namespace

static int execute_kind(pp_scale_plan *P, pp_scale_plan::Kind kind, const pp_frames *src, const pp_frames *dst,
                        int nframes, void *stream) {
    using namespace pp;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int sbytes = P->si.depth > 8 ? 2 : 1;
    switch (kind) {
    case pp_scale_plan::COPY: {
        const int dbytes = P->di.depth > 8 ? 2 : 1;
        for (int p = 0; p < 3; ++p) {
            const int w = p ? P->csw : P->sw, h = p ? P->csh : P->sh;
            dim3 grid((w + 2047) / 2048, h, nframes);
            hipLaunchKernelGGL(copy_widen_kernel, grid, dim3(256), 0, st, (const uint8_t *)src->data[p],
                               src->linesize[p], src->frame_stride[p], sbytes, (uint8_t *)dst->data[p],
                               dst->linesize[p], dst->frame_stride[p], dbytes, w, h, P->di.depth - P->si.depth);
        }
        PP_HIP(hipGetLastError());
        return PP_OK;
    }
    case pp_scale_plan::INTERLEAVE: {
        dim3 grid(((P->sw + 1) / 2 + 1023) / 1024, P->sh, nframes);
        hipLaunchKernelGGL(interleave_uyvy_kernel, grid, dim3(256), 0, st, (const uint8_t *)src->data[0],
                           (const uint8_t *)src->data[1], (const uint8_t *)src->data[2], src->linesize[0],
                           src->linesize[1], src->linesize[2], src->frame_stride[0], src->frame_stride[1],
                           src->frame_stride[2], (uint8_t *)dst->data[0], dst->linesize[0], dst->frame_stride[0],
                           P->sw, P->sh);
        PP_HIP(hipGetLastError());
        return PP_OK;
    }
    case pp_scale_plan::GENERIC:
        return launch_generic(P, src, dst, nframes, st, P->di.depth, true);
    case pp_scale_plan::CHAIN: {
        bool vsrc = true;
        for (int p = 0; p < 3; ++p) vsrc &= aligned(src->data[p], src->linesize[p], nframes > 1 ? src->frame_stride[p] : 0, 16);
        if (P->chain_fused && vsrc) return launch_chain(P, src, dst, nframes, st);
        // two launches through a yuv420p scratch batch (plan-owned: one stream at a time)
        const int64_t yb = (int64_t)P->dw * P->dh, cb = (int64_t)P->cdw * P->cdh;
        const int64_t per = ((yb + 15) & ~int64_t(15)) + 2 * ((cb + 15) & ~int64_t(15));
        if (P->scratch_frames < nframes) {
            if (P->scratch) PP_HIP(hipFree(P->scratch));
            P->scratch = nullptr;
            P->scratch_frames = 0;
            PP_HIP(hipMalloc(&P->scratch, per * nframes));
            P->scratch_frames = nframes;
        }
        uint8_t *s = static_cast<uint8_t *>(P->scratch);
        const int64_t ys = (yb + 15) & ~int64_t(15), cs = (cb + 15) & ~int64_t(15);
        pp_frames tmp{};
        tmp.data[0] = s; tmp.data[1] = s + ys * nframes; tmp.data[2] = s + (ys + cs) * nframes;
        tmp.linesize[0] = P->dw; tmp.linesize[1] = tmp.linesize[2] = P->cdw;
        tmp.frame_stride[0] = ys; tmp.frame_stride[1] = tmp.frame_stride[2] = cs;
        const int rc = execute_kind(P, P->first_kind, src, &tmp, nframes, stream);
        if (rc) return rc;
        return pp_scale_execute(P->stage2, &tmp, dst, nframes, stream);
    }
    case pp_scale_plan::GENERIC_UYVY: {
        bool vsrc = true;
        for (int p = 0; p < 3; ++p) vsrc &= aligned(src->data[p], src->linesize[p], nframes > 1 ? src->frame_stride[p] : 0, 16);
        if (P->fast_hw && vsrc) return launch_packed(P, src, dst, nframes, st);
        // yuv2packedX: planar 8-bit 4:2:2 (flat rounding) then interleave
        const int64_t yb = (int64_t)P->dw * P->dh, cb = (int64_t)P->cdw * P->cdh;
        const int64_t per = yb + 2 * cb;
        if (P->scratch_frames < nframes) {
            if (P->scratch) PP_HIP(hipFree(P->scratch));
            P->scratch = nullptr;
            PP_HIP(hipMalloc(&P->scratch, per * nframes));
            P->scratch_frames = nframes;
        }
        uint8_t *s = static_cast<uint8_t *>(P->scratch);
        pp_frames tmp{};
        tmp.data[0] = s; tmp.data[1] = s + yb * nframes; tmp.data[2] = s + (yb + cb) * nframes;
        tmp.linesize[0] = P->dw; tmp.linesize[1] = tmp.linesize[2] = P->cdw;
        tmp.frame_stride[0] = yb; tmp.frame_stride[1] = tmp.frame_stride[2] = cb;
        // the packed path rounds with 1<<18 and never dithers
        int rc = launch_generic(P, src, &tmp, nframes, st, 8, false);
        if (rc) return rc;
        dim3 grid(((P->dw + 1) / 2 + 1023) / 1024, P->dh, nframes);
        hipLaunchKernelGGL(interleave_uyvy_kernel, grid, dim3(256), 0, st, (const uint8_t *)tmp.data[0],
                           (const uint8_t *)tmp.data[1], (const uint8_t *)tmp.data[2], tmp.linesize[0],
                           tmp.linesize[1], tmp.linesize[2], tmp.frame_stride[0], tmp.frame_stride[1],
                           tmp.frame_stride[2], (uint8_t *)dst->data[0], dst->linesize[0], dst->frame_stride[0],
                           P->dw, P->dh);
        PP_HIP(hipGetLastError());
        return PP_OK;
    }
    }
    PP_FAIL(PP_ERR_INVALID, "bad plan kind");
}

extern "C" int pp_scale_execute(pp_scale_plan *P, const pp_frames *src, const pp_frames *dst, int nframes,
                                void *stream) {
    if (!P || !src || !dst || nframes < 0) PP_FAIL(PP_ERR_INVALID, "null argument");
    if (!P->ctx) PP_FAIL(PP_ERR_INVALID, "host-only plan (created without a context) cannot execute");
    if (nframes == 0) return PP_OK;
    PP_HIP(hipSetDevice(P->ctx->device));
    return execute_kind(P, P->kind, src, dst, nframes, stream);
}
