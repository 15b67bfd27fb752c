// P.910 SI/TI (spec PP-SITI-1) on gfx950.
//
// New feature behind util/SRC_analysis.py:120-147 (analyse_src) and
// util/complexity_classification.py:50-69 (get_difficulty); the reference
// itself has no SI/TI code.
//
//   SI_n = std over rows 1..H-2, cols 1..W-2 of sqrt(Gx^2 + Gy^2)  (Sobel 3x3)
//   TI_n = std over the full frame of Y_n - Y_{n-1}                (n >= 1)
//
// Layout: a workgroup (256 lanes, 4 waves) owns a 1984-px x 16-row band of the
// frame (4 x 496 px; lanes 0 and 63 of a wave are halo lanes) and walks a
// contiguous chunk of frames.  Each lane holds 8 adjacent pixels
// of a row (one 16-B or 8-B load), gets its left/right neighbours by lane
// shuffles (global loads only at wave edges), and slides a 3-row window down
// the band, so every pixel of the band is read from HBM once per frame; the
// previous frame's band (TI) stays in registers (16 rows x 8 px packed in 64
// VGPRs); only the two halo rows are read twice, the second time from L2
// (the neighbouring band runs the same frames on the same XCD, see siti_kernel).
// Precision: |G| = sqrt in fp32; per lane and frame the shifted sums
// S1 = sum(|G| - K), S2 = sum(|G| - K)^2 in fp32, K being one of the lane's own
// samples of that frame (so S2 - S1^2/n cancels at most ~n eps, ~1e-5 relative,
// and a constant-magnitude frame gives exactly 0), merged across lanes, waves
// and bands in fp64 (Chan et al.).
// Moments: SI keeps (count, mean, M2) of |G| per wave (from the lanes' shifted
// sums, so no E[x^2]-mean^2 cancellation); TI keeps sum(d) and
// sum(d^2) exact in 64-bit integers.  Per (frame, band) partials are written
// without atomics and reduced in a fixed order by siti_finalize, so results
// are bit-reproducible.
// Bound: VALU, not HBM -- the interior frame loop is ~1660 VALU instructions
// per wave and frame for 8 x 16 pixels a lane (per pixel: two op_sel'd
// v_pk_mad_i16 build (h1, h2), two more give (gx, gy), one v_dot2 |G|^2, one
// v_sqrt_f32; TI by v_dot2), 0.63-0.65 ms on config 2
// (profiles/r2/siti_experiments.md).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "common.hpp"
#include "device.hpp"

namespace pp {

constexpr int kBand = 16;
constexpr int kLanePx = 8;
constexpr int kWaveSpan = 62 * kLanePx;  // 496 px per wave: lanes 0 and 63 are halo lanes
constexpr int kSpan = 4 * kWaveSpan;     // 1984 px per workgroup
constexpr int kOob = kOobOff;

struct SitiPartial {
    double mean;   // mean of |G| over n samples
    double m2;     // sum (|G| - mean)^2
    int64_t n;     // Sobel samples
    int64_t d1;    // sum (cur - prev)
    uint64_t d2;   // sum (cur - prev)^2
    int64_t pad;
};

// Chan et al. merge of (n, mean, M2) statistics.
__device__ inline void chan_merge(int64_t &n, double &mean, double &m2, int64_t nb, double meanb, double m2b) {
    if (nb == 0) return;
    if (n == 0) { n = nb; mean = meanb; m2 = m2b; return; }
    const int64_t nn = n + nb;
    const double delta = meanb - mean;
    const double fb = static_cast<double>(nb) / static_cast<double>(nn);
    mean += delta * fb;
    m2 += m2b + delta * delta * static_cast<double>(n) * fb;
    n = nn;
}

// One row of a lane's 8 pixels in load format: 4 dwords (u16) or 2 (u8).
template <typename T>
struct Row {
    static constexpr int N = sizeof(T) == 2 ? 4 : 2;
    uint32_t w[N];
    __device__ int px(int e) const {
        if constexpr (sizeof(T) == 2) return (w[e >> 1] >> (16 * (e & 1))) & 0xffff;
        else return (w[e >> 2] >> (8 * (e & 3))) & 0xff;
    }
};

// Issue the load of one row (bounds-checked buffer load; kOob reads 0).
template <typename T>
__device__ inline void issue_row(Row<T> &r, __amdgpu_buffer_rsrc_t rs, int off) {
    if constexpr (sizeof(T) == 2) {
        const auto q = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
        __builtin_memcpy(r.w, &q, 16);
    } else {
        const auto q = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0);
        __builtin_memcpy(r.w, &q, 8);
    }
}

typedef int16_t v2i16 __attribute__((ext_vector_type(2)));
typedef uint16_t v2u16 __attribute__((ext_vector_type(2)));
typedef float v2f32 __attribute__((ext_vector_type(2)));

// packed 16-bit lane-pair arithmetic (v_pk_add_u16 / v_pk_sub_i16)
__device__ inline uint32_t pk_add(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2u16, a) + __builtin_bit_cast(v2u16, b));
}
__device__ inline uint32_t pk_sub(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2i16, a) - __builtin_bit_cast(v2i16, b));
}
// 2 * a + b per 16-bit half in one v_pk_mad_u16 (wraps like the int16 values it
// holds; the compiler splits a * 2 + b into a shift and an add)
__device__ inline uint32_t pk_2a_plus_b(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_pk_mad_u16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(0x00020002u), "v"(b));
    return r;
}
// v_pk_mad_i16 with half selects: per pixel, the H pass builds the pair
// R = (right - left, left + 2 centre + right) straight from the packed pixel
// registers (op_sel broadcasts a half, no v_perm / v_alignbit), and the V pass
// G = (gx, gy) = Ra * (1, -1) + 2 * Rb.lo + Rc from three rows of R -- so
// |G|^2 is one v_dot2 of G with itself.  Constants in SGPRs (VOP3P takes no
// literal on gfx9).
#define PP_PKMAD(SEL, SELHI)                                                                 \
    [](uint32_t a, uint32_t b, uint32_t c) {                                                 \
        uint32_t r;                                                                          \
        asm("v_pk_mad_i16 %0, %1, %2, %3 op_sel:" SEL " op_sel_hi:" SELHI                    \
            : "=v"(r) : "v"(a), "s"(b), "v"(c));                                             \
        return r;                                                                            \
    }
constexpr uint32_t kC02 = 0x00020000u;   // (0, 2)
constexpr uint32_t kCM11 = 0x0001ffffu;  // (-1, 1)
constexpr uint32_t kC20 = 0x00000002u;   // (2, 0)
constexpr uint32_t kC1M1 = 0xffff0001u;  // (1, -1)

// gx^2 + gy^2 of one (gx, gy) pair: the VOP3P form with an inline-constant
// accumulator (the compiler's v_dot2c form needs a zeroed destination copy)
__device__ inline int sq_norm(v2i16 p) {
    int r;
    asm("v_dot2_i32_i16 %0, %1, %1, 0" : "=v"(r) : "v"(p));
    return r;
}
__device__ inline v2f32 pk_fma(v2f32 a, v2f32 b, v2f32 c) { return __builtin_elementwise_fma(a, b, c); }

// A lane's 8 pixels as four u16 pairs (v[2k], v[2k+1]).
template <typename T>
__device__ inline void to_pairs(const Row<T> &r, uint32_t w[4]) {
    if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = r.w[k];
    } else {
        w[0] = __builtin_amdgcn_perm(0u, r.w[0], 0x0c010c00u);
        w[1] = __builtin_amdgcn_perm(0u, r.w[0], 0x0c030c02u);
        w[2] = __builtin_amdgcn_perm(0u, r.w[1], 0x0c010c00u);
        w[3] = __builtin_amdgcn_perm(0u, r.w[1], 0x0c030c02u);
    }
}

// Wave-wide sums without LDS round trips: quad permutes, the row mirrors,
// then gfx950's 16- and 32-lane swaps.  Every step adds the same pair of
// values on both lanes of the pair (IEEE addition commutes exactly), so all
// lanes end with identical bits and the order is fixed: reproducible.
template <int CTRL>
__device__ inline uint32_t dpp32(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ inline double dpp64(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint64_t r = (uint64_t)dpp32<CTRL>((uint32_t)b) | ((uint64_t)dpp32<CTRL>((uint32_t)(b >> 32)) << 32);
    return __builtin_bit_cast(double, r);
}
// the two values a lane's row pair (16-lane rows) / wave half pair hold
__device__ inline void swap16(uint32_t v, uint32_t &a, uint32_t &b) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    a = r[0]; b = r[1];
}
__device__ inline void swap32(uint32_t v, uint32_t &a, uint32_t &b) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    a = r[0]; b = r[1];
}
template <typename V>
__device__ inline V row_sum(V v) {  // sum over each 16-lane row
    if constexpr (sizeof(V) == 8) {
        v += dpp64<0xB1>(v);   // quad_perm [1,0,3,2]
        v += dpp64<0x4E>(v);   // quad_perm [2,3,0,1]
        v += dpp64<0x141>(v);  // row_half_mirror
        v += dpp64<0x140>(v);  // row_mirror
    } else {
        v += (V)dpp32<0xB1>((uint32_t)v);
        v += (V)dpp32<0x4E>((uint32_t)v);
        v += (V)dpp32<0x141>((uint32_t)v);
        v += (V)dpp32<0x140>((uint32_t)v);
    }
    return v;
}
__device__ inline double wave_sum_f64(double v) {
    v = row_sum(v);
    uint64_t b = __builtin_bit_cast(uint64_t, v);
    uint32_t l0, l1, h0, h1;
    swap16((uint32_t)b, l0, l1);
    swap16((uint32_t)(b >> 32), h0, h1);
    v = __builtin_bit_cast(double, (uint64_t)l0 | ((uint64_t)h0 << 32)) +
        __builtin_bit_cast(double, (uint64_t)l1 | ((uint64_t)h1 << 32));
    b = __builtin_bit_cast(uint64_t, v);
    swap32((uint32_t)b, l0, l1);
    swap32((uint32_t)(b >> 32), h0, h1);
    return __builtin_bit_cast(double, (uint64_t)l0 | ((uint64_t)h0 << 32)) +
           __builtin_bit_cast(double, (uint64_t)l1 | ((uint64_t)h1 << 32));
}
__device__ inline int wave_sum_i32(int v) {
    v = row_sum(v);
    uint32_t a, b;
    swap16((uint32_t)v, a, b);
    swap32(a + b, a, b);
    return (int)(a + b);
}
// sum of u32 values whose 32-lane sums fit in 32 bits; the last step in 64
__device__ inline uint64_t wave_sum_u32_wide(uint32_t v) {
    v = row_sum(v);
    uint32_t a, b;
    swap16(v, a, b);
    swap32(a + b, a, b);
    return (uint64_t)a + (uint64_t)b;
}

// Window of a workgroup's band: rows y0-1 .. y0+kBand of one frame, held as
// raw load registers.  Row ri's registers are reloaded with the NEXT frame's
// row ri right after frame f consumes them, so a whole frame of loads is in
// flight while the current one is computed, with no extra registers and no
// branches around the loads.  The previous frame's band (TI) stays in
// registers too, so every pixel is read from HBM once (plus the two halo rows).
//
// INTERIOR (every band but the first and the last): all 18 window rows lie in
// the frame and all 16 Sobel centres are valid, so the unrolled row loop has
// no per-row conditions at all (they cost SGPRs, spilled to VGPR lanes, and a
// branch per row).  Lanes outside the frame and the halo lanes carry no TI
// samples: their TI sums are dropped once per frame instead of masking every
// pixel; only a lane straddling a ragged right edge (RAGGED: W % 8 != 0) masks
// its pixels.  The next frame's rows are read through a descriptor of 0 bytes
// after the range's last frame (no traffic, no per-row liveness test).
template <typename T, bool INTERIOR, bool RAGGED>
__device__ __forceinline__ void siti_range(const uint8_t *frames, int64_t ls, int64_t fs, const uint8_t *prev, int W,
                                          int H, int tiles_x, int tile, int f0, int f1, SitiPartial *part) {
    constexpr int NR = kBand + 2;
    const int bands = (H + kBand - 1) / kBand;
    const int tx = tile % tiles_x, band = tile / tiles_x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // lanes 1..62 own 8 pixels each; lanes 0 and 63 load the pixels just left
    // and right of the wave's span, so every neighbour comes from a shuffle
    const int x = tx * kSpan + wave * kWaveSpan + (lane - 1) * kLanePx;
    const bool halo = lane == 0 || lane == 63;
    const int y0 = band * kBand, y1 = min(H, y0 + kBand);
    // lane-relative valid Sobel columns [lo, hi] (empty for halo lanes)
    const int sobel_lo = halo ? kLanePx : 1 - x, sobel_hi = halo ? -1 : W - 2 - x;
    // TI: lanes whose 8 pixels are all frame pixels the wave accounts for; the
    // straddling lane of a ragged edge masks per pixel
    const bool ti_lane = !halo && x >= 0 && x < W;

    // a row load straddling num_records reads 0 as a whole: the last row counts
    // up to its load-granule-rounded width, which lies inside the (aligned) pitch
    constexpr int G = kLanePx * sizeof(T);
    const int frame_bytes = (int)((int64_t)(H - 1) * ls + min(ls, ((int64_t)W * sizeof(T) + G - 1) / G * G));
    const bool x_in = x >= 0 && x < W;  // lane 0 of the first wave sits left of the frame
    // row r of a frame at lane offset voff + r * ls (unsigned: row -1 and rows
    // >= H fall outside num_records and read 0; so does every row of a lane
    // outside the frame, which starts at kOob)
    const uint32_t voff = x_in ? (uint32_t)(x * (int)sizeof(T)) : (uint32_t)kOob;
    const uint32_t uls = (uint32_t)ls;
    auto row_off = [&](int r) { return voff + (uint32_t)r * uls; };

    Row<T> raw[NR], pv[kBand];
    // previous frame's band
    const uint8_t *pfirst = f0 > 0 ? frames + (f0 - 1) * fs : prev;
    {
        const auto prs = uniform_rsrc(pfirst ? pfirst : frames, pfirst ? frame_bytes : 0);
#pragma unroll
        for (int i = 0; i < kBand; ++i) issue_row<T>(pv[i], prs, row_off(y0 + i));
    }
    // first frame's window
    {
        const auto crs = uniform_rsrc(frames + (int64_t)f0 * fs, frame_bytes);
#pragma unroll
        for (int ri = 0; ri < NR; ++ri) issue_row<T>(raw[ri], crs, row_off(y0 - 1 + ri));
    }

    // per-lane constants of the packed formulation
    uint32_t tmask[4];  // TI: 0xffff per pixel this lane accounts for (RAGGED only)
    v2f32 vm[4];        // Sobel: 1.0 per valid Sobel column, else 0
    int rc = 0;         // valid Sobel columns of this lane
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int e0 = 2 * k, e1 = 2 * k + 1;
        const bool t0 = x + e0 < W, t1 = x + e1 < W;
        tmask[k] = (t0 ? 0xffffu : 0u) | (t1 ? 0xffff0000u : 0u);
        const bool s0 = e0 >= sobel_lo && e0 <= sobel_hi, s1 = e1 >= sobel_lo && e1 <= sobel_hi;
        vm[k] = v2f32{s0 ? 1.f : 0.f, s1 ? 1.f : 0.f};
        rc += s0 + s1;
    }
    // valid Sobel rows c of the band (the same for every frame) and whether
    // the band's first window row (ri == 2, c = y0) is one of them
    const int sobel_rows = max(0, min(y1 - 1, H - 2) - max(y0, 1) + 1);
    const bool row2_valid = y0 >= 1 && y0 < y1 && y0 <= H - 2;
    const double n_lane = static_cast<double>(rc) * sobel_rows;
    // the wave's Sobel sample count: the same for every frame
    const double cnt_w = wave_sum_f64(n_lane);
    // the lane's first valid Sobel column supplies the frame's shift K
    const int kpick = halo ? 0 : max(0, min(kLanePx - 1, sobel_lo));
    const uint32_t ones = 0x00010001u;

    // Frame f's lane sums are reduced across the wave in the middle of frame
    // f+1's rows (the range's last frame after the loop), so the reduction's
    // dependent chains overlap independent row work.  fp64 in a fixed order:
    // sum (n K + S1) -> mean_w, then sum (x - mean_w)^2 = sum (S2 + 2 dK S1 +
    // n dK^2), dK = K - mean_w; TI moments as integers (|sum d| < 2^31 over a
    // wave; sum d^2 of 32 lanes < 2^32, the last step in 64 bits).  The store
    // is a buffer store whose offset is out of range on every lane but lane 0
    // of a pending frame: no branch, the frame loop stays one basic block.
    auto reduce_store = [&](int fq, bool live, float Kq, double l1, double l2, int q1, uint32_t q2, bool hp) {
        const double sum = wave_sum_f64(n_lane * static_cast<double>(Kq) + l1);
        const double mean_w = cnt_w > 0.0 ? sum / cnt_w : 0.0;
        const double dk = static_cast<double>(Kq) - mean_w;
        const double m2 = wave_sum_f64(l2 + 2.0 * dk * l1 + n_lane * dk * dk);
        const int d1 = wave_sum_i32(ti_lane ? q1 : 0);
        const uint64_t d2w = wave_sum_u32_wide(ti_lane ? q2 : 0u);
        const int64_t idx = ((int64_t)max(fq, 0) * tiles_x * bands + tile) * 4 + wave;
        const auto prs = uniform_rsrc(part + idx, (int)sizeof(SitiPartial));
        const uint32_t o = (live && lane == 0) ? 0u : static_cast<uint32_t>(kOob);
        const uint64_t n64 = static_cast<uint64_t>(static_cast<int64_t>(cnt_w));
        const uint64_t d164 = hp ? static_cast<uint64_t>(static_cast<int64_t>(d1)) : 0u;
        const uint64_t d264 = hp ? d2w : 0u;
        const uint64_t mb = __builtin_bit_cast(uint64_t, mean_w), qb = __builtin_bit_cast(uint64_t, m2);
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        auto pack = [](uint64_t a, uint64_t b) {
            return u32x4{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
        };
        __builtin_amdgcn_raw_buffer_store_b128(pack(mb, qb), prs, o, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(pack(n64, d164), prs, o + 16, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(pack(d264, 0), prs, o + 32, 0, 0);
    };
    bool pend = false, p_hp = false;
    float p_K = 0.f;
    double p_l1 = 0.0, p_l2 = 0.0;
    int p_d1 = 0;
    uint32_t p_d2 = 0;

    for (int f = f0; f < f1; ++f) {
        const bool has_prev = f > 0 || prev != nullptr;
        const bool nlive = f + 1 < f1;
        const auto nrs = uniform_rsrc(frames + (int64_t)(nlive ? f + 1 : f) * fs, nlive ? frame_bytes : 0);
        // the row offsets are frame-invariant: recompute them per frame (one
        // SALU op a row) instead of letting 18 hoisted values spill
        uint32_t fls = uls;
        asm volatile("" : "+s"(fls));
        // shifted moments of |G|: x = |G| - K over the lane's valid columns,
        // S1 = sum x, S2 = sum x^2 (K = one of the lane's own samples, so a
        // constant-magnitude frame gives x = 0 exactly and SI = 0 exactly)
        float K = 0.f;
        v2f32 nkvm[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};  // -K * valid mask
        v2f32 s1 = {0.f, 0.f}, s2 = {0.f, 0.f};
        int d1s = 0;        // |sum d| <= 16 rows * 8 px * 1023
        uint32_t d2s = 0;   // sum d^2 <= 16 * 8 * 1023^2 < 2^32
        uint32_t Ra[kLanePx], Rb[kLanePx];  // (h1, h2) of the two rows above
#pragma unroll
        for (int ri = 0; ri < NR; ++ri) {
            const int r = y0 - 1 + ri;
            const bool band = ri >= 1 && ri <= kBand;
            const int bi = ri - 1;
            uint32_t w[4];
            to_pairs<T>(raw[ri], w);
            // neighbours: the last pixel of the lane below, the first of the lane above
            // (DPP wave shifts; only halo lanes see the wave's ends)
            const uint32_t wl = __builtin_amdgcn_mov_dpp(w[3], 0x138, 0xf, 0xf, true);  // wave_shr:1
            const uint32_t wr = __builtin_amdgcn_mov_dpp(w[0], 0x130, 0xf, 0xf, true);  // wave_shl:1
            // R[i] = (h1, h2) of pixel i: h1 = right - left, h2 = left + 2 v + right
            uint32_t R[kLanePx];
            {
                const auto mad_t0 = PP_PKMAD("[0,0,1]", "[0,1,1]");  // (v[2k+1], 2 v[2k] + v[2k+1])
                const auto mad_r0 = PP_PKMAD("[1,0,0]", "[1,1,1]");  // + (-1, 1) * v[2k-1]
                const auto mad_t1 = PP_PKMAD("[1,0,0]", "[1,1,0]");  // (v[2k+2], 2 v[2k+1] + v[2k+2])
                const auto mad_r1 = PP_PKMAD("[0,0,0]", "[0,1,1]");  // + (-1, 1) * v[2k]
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t lft = k ? w[k - 1] : wl, rgt = k < 3 ? w[k + 1] : wr;
                    R[2 * k] = mad_r0(lft, kCM11, mad_t0(w[k], kC02, w[k]));
                    R[2 * k + 1] = mad_r1(w[k], kCM11, mad_t1(w[k], kC02, rgt));
                }
            }
            // TI on the band rows against the previous frame's band
            if (band) {
                if (INTERIOR || r < y1) {
                    uint32_t q[4];
                    to_pairs<T>(pv[bi], q);
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        uint32_t dd = pk_sub(w[k], q[k]);
                        if constexpr (RAGGED) dd &= tmask[k];
                        const v2i16 d = __builtin_bit_cast(v2i16, dd);
                        d1s = __builtin_amdgcn_sdot2(d, __builtin_bit_cast(v2i16, ones), d1s, false);
                        d2s = static_cast<uint32_t>(__builtin_amdgcn_sdot2(d, d, static_cast<int>(d2s), false));
                    }
                }
                pv[bi] = raw[ri];  // (swapping raw/pv roles per frame instead: 178 VGPR spills)
            }
            // Sobel centred on row c = r - 1 (rows c-1, c, c+1 are in the window)
            const int c = r - 1;
            if (ri >= 2 && (INTERIOR || (c < y1 && c >= 1 && c <= H - 2))) {
                v2f32 mag[4];
                const auto mad_in = PP_PKMAD("[0,0,0]", "[1,1,1]");
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    int g[2];
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const int i = 2 * k + e;
                        // G = (Ra.lo + 2 Rb.lo + Rc.lo, Rc.hi - Ra.hi) = (gx, gy), |.| <= 4092
                        const uint32_t G = mad_in(Ra[i], kC1M1, mad_in(Rb[i], kC20, R[i]));
                        g[e] = sq_norm(__builtin_bit_cast(v2i16, G));
                    }
                    mag[k] = v2f32{__fsqrt_rn(static_cast<float>(g[0])), __fsqrt_rn(static_cast<float>(g[1]))};
                }
                // first valid Sobel row of the band
                if (INTERIOR ? ri == 2 : (ri == 2 || (ri == 3 && !row2_valid))) {
                    float k = mag[0].x;
#pragma unroll
                    for (int e = 1; e < kLanePx; ++e) k = kpick == e ? ((e & 1) ? mag[e >> 1].y : mag[e >> 1].x) : k;
                    K = k;
                    const v2f32 nk = {-K, -K};
#pragma unroll
                    for (int j = 0; j < 4; ++j) nkvm[j] = vm[j] * nk;
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const v2f32 xv = pk_fma(mag[j], vm[j], nkvm[j]);  // (|G| - K) on valid columns, else 0
                    s1 += xv;
                    s2 = pk_fma(xv, xv, s2);
                }
            }
#pragma unroll
            for (int i = 0; i < kLanePx; ++i) {
                Ra[i] = Rb[i];
                Rb[i] = R[i];
            }
            // this row is consumed: start loading the next frame's row ri into it
            issue_row<T>(raw[ri], nrs, voff + (uint32_t)r * fls);
            if (ri == 6) reduce_store(f - 1, pend, p_K, p_l1, p_l2, p_d1, p_d2, p_hp);
        }
        pend = true;
        p_hp = has_prev;
        p_K = K;
        p_l1 = static_cast<double>(s1.x) + static_cast<double>(s1.y);
        p_l2 = static_cast<double>(s2.x) + static_cast<double>(s2.y);
        p_d1 = d1s;
        p_d2 = d2s;
    }
    if (pend) reduce_store(f1 - 1, true, p_K, p_l1, p_l2, p_d1, p_d2, p_hp);
}

// 1-D grid sized to the resident workgroup slots.  The frames are cut into
// chunks of `fchunk` and the (chunk, tile) units are numbered chunk-major;
// workgroup L takes units L, L + G, L + 2G, ...  So the workgroups running at
// any moment hold vertically adjacent bands of the SAME frames, and with the
// XCD-aware numbering (consecutive L on one XCD) a band's two halo rows are
// read from HBM by one neighbour and hit that XCD's L2 for the other.  The
// host picks fchunk so that the rounds of units fill the slots (see pp_siti).
template <typename T, bool RAGGED>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void siti_kernel(
    const uint8_t *frames, int64_t ls, int64_t fs, int nframes, const uint8_t *prev, int W, int H, int tiles_x,
    int ntiles, int fchunk, SitiPartial *part) {
    const int chunks = (nframes + fchunk - 1) / fchunk;
    const int64_t total = (int64_t)ntiles * chunks;
    for (int64_t u = xcd_remap(blockIdx.x, gridDim.x); u < total; u += gridDim.x) {
        const int chunk = (int)(u / ntiles);
        const int tile = (int)(u - (int64_t)chunk * ntiles);
        const int f0 = chunk * fchunk, f1 = min(nframes, f0 + fchunk);
        const int y0 = tile / tiles_x * kBand;
        if (y0 >= 1 && y0 + kBand + 1 <= H)
            siti_range<T, true, RAGGED>(frames, ls, fs, prev, W, H, tiles_x, tile, f0, f1, part);
        else
            siti_range<T, false, RAGGED>(frames, ls, fs, prev, W, H, tiles_x, tile, f0, f1, part);
    }
}

// One workgroup per frame: each lane merges a strided subset of the partials,
// then a fixed-shape LDS tree -- the order never depends on timing, so the
// result is bit-reproducible.
__global__ __launch_bounds__(256) void siti_finalize(const SitiPartial *part, int nframes, int nparts, int W, int H,
                                                     int has_prev, double scale, double *si, double *ti) {
    __shared__ double s_mean[256], s_m2[256];
    __shared__ int64_t s_n[256], s_d1[256];
    __shared__ uint64_t s_d2[256];
    const int f = blockIdx.x, t = threadIdx.x;
    double mean = 0.0, m2 = 0.0;
    int64_t n = 0, d1 = 0;
    uint64_t d2 = 0;
    for (int i = t; i < nparts; i += 256) {
        const SitiPartial &p = part[(int64_t)f * nparts + i];
        chan_merge(n, mean, m2, p.n, p.mean, p.m2);
        d1 += p.d1; d2 += p.d2;
    }
    s_mean[t] = mean; s_m2[t] = m2; s_n[t] = n; s_d1[t] = d1; s_d2[t] = d2;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (t < o) {
            chan_merge(s_n[t], s_mean[t], s_m2[t], s_n[t + o], s_mean[t + o], s_m2[t + o]);
            s_d1[t] += s_d1[t + o];
            s_d2[t] += s_d2[t + o];
        }
        __syncthreads();
    }
    if (t) return;
    // scale: 1, or 2^-(bitdepth-8) with PP_SITI_NORMALIZE (an exact power of two)
    si[f] = s_n[0] ? sqrt(s_m2[0] / static_cast<double>(s_n[0])) * scale : 0.0;
    if (f == 0 && !has_prev) {
        ti[f] = __builtin_nan("");
    } else {
        const int64_t np = static_cast<int64_t>(W) * H;
        const __int128 num = static_cast<__int128>(np) * static_cast<__int128>(s_d2[0]) -
                             static_cast<__int128>(s_d1[0]) * static_cast<__int128>(s_d1[0]);
        ti[f] = sqrt(static_cast<double>(num)) / static_cast<double>(np) * scale;
    }
}

}  // namespace pp

using namespace pp;

extern "C" int pp_siti(pp_ctx *ctx, int bitdepth, int w, int h, const void *luma, int64_t linesize,
                       int64_t frame_stride, int nframes, const void *prev, double *si, double *ti, void *stream) {
    return pp_siti_ex(ctx, bitdepth, w, h, luma, linesize, frame_stride, nframes, prev, si, ti, 0, stream);
}

extern "C" int pp_siti_ex(pp_ctx *ctx, int bitdepth, int w, int h, const void *luma, int64_t linesize,
                          int64_t frame_stride, int nframes, const void *prev, double *si, double *ti, int flags,
                          void *stream) {
    if (flags & ~PP_SITI_NORMALIZE) PP_FAIL(PP_ERR_INVALID, "siti flags 0x%x", flags);
    if (!ctx || !luma || !si || !ti || nframes < 0) PP_FAIL(PP_ERR_INVALID, "null argument");
    if (bitdepth != 8 && bitdepth != 10) PP_FAIL(PP_ERR_INVALID, "bit depth %d (8 or 10)", bitdepth);
    if (w < 3 || h < 3) PP_FAIL(PP_ERR_INVALID, "frame %dx%d too small for Sobel", w, h);
    if (nframes == 0) return PP_OK;
    hipStream_t st = static_cast<hipStream_t>(stream);
    PP_HIP(hipSetDevice(ctx->device));
    const int bytes = bitdepth > 8 ? 2 : 1;
    const int tiles_x = (w + kSpan - 1) / kSpan;
    const int bands = (h + kBand - 1) / kBand;
    const int ntiles = tiles_x * bands;
    const bool ragged = (w % kLanePx) != 0;
    using KFn = void (*)(const uint8_t *, int64_t, int64_t, int, const uint8_t *, int, int, int, int, int,
                         SitiPartial *);
    const KFn k = bytes == 2 ? (ragged ? siti_kernel<uint16_t, true> : siti_kernel<uint16_t, false>)
                             : (ragged ? siti_kernel<uint8_t, true> : siti_kernel<uint8_t, false>);
    const void *kfn = reinterpret_cast<const void *>(k);
    // one wave of resident workgroups (a partial second wave would idle most of
    // the chip), each walking an equal share of the (tile, frame) units
    int dev_cus = 0, per_cu = 0;
    PP_HIP(hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    PP_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, 256, 0));
    const int64_t slots = std::max(1, dev_cus * std::max(1, per_cu));
    // frames per chunk: for R = 1..8 rounds of units over the slots, the
    // longest chunk that still fits R rounds; keep the R with the shortest
    // makespan (R * fchunk frames, plus ~1 frame of pipeline fill per round)
    int fchunk = nframes;
    {
        double best = 1e300;
        for (int R = 1; R <= 8; ++R) {
            const int K = (int)std::max<int64_t>(1, std::min<int64_t>(nframes, R * slots / ntiles));
            const int fc = (nframes + K - 1) / K;
            const int64_t units = (int64_t)ntiles * ((nframes + fc - 1) / fc);
            const int64_t rounds = (units + std::min(slots, units) - 1) / std::min(slots, units);
            const double cost = (double)rounds * (fc + 1);
            if (cost < best) { best = cost; fchunk = fc; }
        }
    }
    const int groups = (int)std::min<int64_t>(slots, (int64_t)ntiles * ((nframes + fchunk - 1) / fchunk));
    // The kernel reads each lane's 8 pixels as one 16-B (8-B) buffer load, so
    // rows must start on that granule; other layouts (odd widths packed
    // contiguously, views into a row) are first repacked on the device into a
    // pitched scratch copy -- one extra read+write, never a second code path.
    const int a = bytes == 2 ? 16 : 8;
    const bool aligned = ((uintptr_t)luma % a == 0) && (linesize % a == 0) && (nframes < 2 || frame_stride % a == 0) &&
                         (!prev || (uintptr_t)prev % a == 0);
    const uint8_t *src = static_cast<const uint8_t *>(luma), *psrc = static_cast<const uint8_t *>(prev);
    int64_t ls = linesize, fs = frame_stride;
    uint8_t *scratch = nullptr;
    if (!aligned) {
        ls = ((int64_t)w * bytes + 15) & ~int64_t(15);
        fs = ls * h;
    }
    // checked before any allocation, so a refused call leaks nothing
    if ((int64_t)(h - 1) * ls + (int64_t)w * bytes >= (int64_t)kOob)
        PP_FAIL(PP_ERR_UNSUPPORTED, "frame of %lld bytes exceeds the 2 GiB buffer range", (long long)(h * ls));
    SitiPartial *part = nullptr;
    PP_HIP(hipMallocAsync((void **)&part, sizeof(SitiPartial) * (size_t)ntiles * 4 * nframes, st));
    if (!aligned) {
        const int nf = nframes + (prev ? 1 : 0);
        const hipError_t e = hipMallocAsync((void **)&scratch, (size_t)(fs * nf), st);
        if (e != hipSuccess) {
            (void)hipFreeAsync(part, st);
            PP_FAIL(PP_ERR_HIP, "siti scratch (%lld bytes): %s", (long long)(fs * nf), hipGetErrorString(e));
        }
        uint8_t *dst = scratch + (prev ? fs : 0);
        if (nframes == 1 || frame_stride == linesize * h) {
            PP_HIP(hipMemcpy2DAsync(dst, ls, luma, linesize, (size_t)w * bytes, (size_t)h * nframes,
                                    hipMemcpyDeviceToDevice, st));
        } else {
            for (int f = 0; f < nframes; ++f)
                PP_HIP(hipMemcpy2DAsync(dst + f * fs, ls, static_cast<const uint8_t *>(luma) + f * frame_stride,
                                        linesize, (size_t)w * bytes, h, hipMemcpyDeviceToDevice, st));
        }
        if (prev)
            PP_HIP(hipMemcpy2DAsync(scratch, ls, prev, linesize, (size_t)w * bytes, h, hipMemcpyDeviceToDevice, st));
        src = dst;
        psrc = prev ? scratch : nullptr;
    }
    hipLaunchKernelGGL(k, dim3(groups), dim3(256), 0, st, src, ls, fs, nframes, psrc, w, h, tiles_x, ntiles, fchunk,
                       part);
    hipLaunchKernelGGL(siti_finalize, dim3(nframes), dim3(256), 0, st, part, nframes, ntiles * 4, w, h,
                       prev != nullptr, (flags & PP_SITI_NORMALIZE) ? 1.0 / (double)(1 << (bitdepth - 8)) : 1.0, si,
                       ti);  // ntiles * 4 wave partials per frame
    PP_HIP(hipGetLastError());
    PP_HIP(hipFreeAsync(part, st));
    if (scratch) PP_HIP(hipFreeAsync(scratch, st));
    return PP_OK;
}
