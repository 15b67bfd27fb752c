// P.910 SI/TI (spec PP-SITI-1) on gfx950.
//
// New feature behind util/SRC_analysis.py:120-147 (analyse_src) and
// util/complexity_classification.py:50-69 (get_difficulty); the reference
// itself has no SI/TI code.
//
//   SI_n = std over rows 1..H-2, cols 1..W-2 of sqrt(Gx^2 + Gy^2)  (Sobel 3x3)
//   TI_n = std over the full frame of Y_n - Y_{n-1}                (n >= 1)
//
// Layout: a workgroup (256 lanes) owns a 2048-px x 16-row band of the frame
// and walks a contiguous chunk of frames.  Each lane holds 8 adjacent pixels
// of a row (one 16-B or 8-B load), gets its left/right neighbours by lane
// shuffles (global loads only at wave edges), and slides a 3-row window down
// the band, so every pixel of the band is read from HBM once per frame; the
// previous frame's band (TI) stays in registers (16 rows x 8 px packed in 64
// VGPRs), only the two halo rows are read twice.
// Precision: |G| = sqrt in fp32 and per-row (mean, M2) in fp32 -- std is
// shift-invariant, so a relative rounding of ~1e-7 per sample moves SI by
// ~1e-7 relative, well inside the 1e-4 tolerance -- merged across rows, lanes
// and bands in fp64 (Chan et al.).
// Moments: SI keeps (count, mean, M2) of |G| -- per-row two-pass statistics
// merged with Chan's parallel update, so a frame of constant gradient
// magnitude gives exactly 0 (E[x^2]-mean^2 would cancel); TI keeps sum(d) and
// sum(d^2) exact in 64-bit integers.  Per (frame, band) partials are written
// without atomics and reduced in a fixed order by siti_finalize, so results
// are bit-reproducible.
#include <cmath>

#include "common.hpp"

namespace pp {

constexpr int kBand = 16;
constexpr int kLanePx = 8;
constexpr int kSpan = 256 * kLanePx;  // 2048 px per workgroup

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

template <typename T>
__device__ inline void load_row(int v[kLanePx], const T *row, int x, int W, bool vec) {
    if (vec && x + kLanePx <= W) {
        if constexpr (sizeof(T) == 2) {
            const uint4 q = *reinterpret_cast<const uint4 *>(row + x);
            v[0] = q.x & 0xffff; v[1] = q.x >> 16; v[2] = q.y & 0xffff; v[3] = q.y >> 16;
            v[4] = q.z & 0xffff; v[5] = q.z >> 16; v[6] = q.w & 0xffff; v[7] = q.w >> 16;
        } else {
            const uint2 q = *reinterpret_cast<const uint2 *>(row + x);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[e] = (q.x >> (8 * e)) & 0xff;
                v[4 + e] = (q.y >> (8 * e)) & 0xff;
            }
        }
    } else {
#pragma unroll
        for (int e = 0; e < kLanePx; ++e) v[e] = (x + e < W) ? static_cast<int>(row[x + e]) : 0;
    }
}

__device__ inline uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Lane-local (n, mean, M2) in fp32, merged with Chan's update.
__device__ inline void chan_merge_f(float &n, float &mean, float &m2, float nb, float meanb, float m2b) {
    const float nn = n + nb;
    const float delta = meanb - mean;
    const float fb = nn > 0.f ? nb / nn : 0.f;
    mean += delta * fb;
    m2 += m2b + delta * delta * n * fb;
    n = nn;
}

template <typename T>
__device__ inline void pack_row(uint32_t pk[4], const int v[kLanePx]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) pk[e] = (uint32_t)v[2 * e] | ((uint32_t)v[2 * e + 1] << 16);
}

template <typename T>
__global__ __launch_bounds__(256) void siti_kernel(const uint8_t *frames, int64_t ls, int64_t fs, int nframes,
                                                   const uint8_t *prev, int W, int H, int tiles_x, int bands,
                                                   int chunk, int vec, SitiPartial *part) {
    __shared__ SitiPartial red[4];
    const int tile = blockIdx.x;  // tx + tiles_x * band
    const int tx = tile % tiles_x, band = tile / tiles_x;
    const int f0 = blockIdx.y * chunk, f1 = min(nframes, f0 + chunk);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x = tx * kSpan + threadIdx.x * kLanePx;
    const int y0 = band * kBand, y1 = min(H, y0 + kBand);
    const bool wave_left = lane == 0, wave_right = lane == 63;
    int valid_px = 0;  // pixels of this lane inside the frame
#pragma unroll
    for (int e = 0; e < kLanePx; ++e) valid_px += (x + e < W);
    int sobel_lo = 1 - x, sobel_hi = W - 2 - x;  // lane-relative valid Sobel columns [lo, hi]

    // previous frame's band, packed 2 samples per register (TI without re-reading HBM)
    uint32_t pv[kBand][4];
    const uint8_t *pfirst = f0 > 0 ? frames + (f0 - 1) * fs : prev;
    if (pfirst) {
#pragma unroll
        for (int i = 0; i < kBand; ++i) {
            int q[kLanePx] = {0, 0, 0, 0, 0, 0, 0, 0};
            if (y0 + i < y1) load_row<T>(q, reinterpret_cast<const T *>(pfirst + (int64_t)(y0 + i) * ls), x, W, vec);
            pack_row<T>(pv[i], q);
        }
    }

    for (int f = f0; f < f1; ++f) {
        const uint8_t *cur = frames + f * fs;
        const bool has_prev = f > 0 || prev != nullptr;
        float n_t = 0.f, mean_t = 0.f, m2_t = 0.f;
        uint64_t d2s = 0;
        int64_t d1s = 0;
        int h1a[kLanePx], h2a[kLanePx], h1b[kLanePx], h2b[kLanePx];
        // rows y0-1 .. y0+kBand, fully unrolled so the band index is a constant
#pragma unroll
        for (int ri = 0; ri < kBand + 2; ++ri) {
            const int r = y0 - 1 + ri;
            int v[kLanePx] = {0, 0, 0, 0, 0, 0, 0, 0};
            int h1[kLanePx], h2[kLanePx];
            if (r >= 0 && r < H) {
                const T *row = reinterpret_cast<const T *>(cur + (int64_t)r * ls);
                load_row<T>(v, row, x, W, vec);
                int left = __shfl_up(v[kLanePx - 1], 1, 64);
                int right = __shfl_down(v[0], 1, 64);
                if (wave_left) left = (x - 1 >= 0 && x - 1 < W) ? static_cast<int>(row[x - 1]) : 0;
                if (wave_right) right = (x + kLanePx < W) ? static_cast<int>(row[x + kLanePx]) : 0;
#pragma unroll
                for (int e = 0; e < kLanePx; ++e) {
                    const int l = e ? v[e - 1] : left;
                    const int rr = e < kLanePx - 1 ? v[e + 1] : right;
                    h1[e] = rr - l;
                    h2[e] = l + 2 * v[e] + rr;
                }
            } else {
#pragma unroll
                for (int e = 0; e < kLanePx; ++e) h1[e] = h2[e] = 0;
            }
            // TI on the band rows, previous frame from registers
            const int bi = ri - 1;
            if (ri >= 1 && ri <= kBand && r < y1) {
                if (has_prev) {
                    int ds = 0;
                    uint32_t dq = 0;
#pragma unroll
                    for (int e = 0; e < kLanePx; ++e) {
                        const int q = (pv[bi][e >> 1] >> (16 * (e & 1))) & 0xffff;
                        const int d = (e < valid_px) ? v[e] - q : 0;
                        ds += d;
                        dq += static_cast<uint32_t>(d * d);
                    }
                    d1s += ds;
                    d2s += dq;
                }
                pack_row<T>(pv[bi], v);
            }
            // Sobel centred on row c = r - 1 (rows c-1, c, c+1 are in the window)
            const int c = r - 1;
            if (ri >= 2 && c < y1 && c >= 1 && c <= H - 2) {
                float mag[kLanePx];
                float rs = 0.f;
                int rc = 0;
#pragma unroll
                for (int e = 0; e < kLanePx; ++e) {
                    const int gx = h1a[e] + 2 * h1b[e] + h1[e];
                    const int gy = h2[e] - h2a[e];
                    const bool ok = e >= sobel_lo && e <= sobel_hi;
                    mag[e] = ok ? __fsqrt_rn(static_cast<float>(gx * gx + gy * gy)) : 0.f;
                    rs += mag[e];
                    rc += ok;
                }
                if (rc) {
                    const float rm = rs / static_cast<float>(rc);
                    float rm2 = 0.f;
#pragma unroll
                    for (int e = 0; e < kLanePx; ++e) {
                        const float dv = mag[e] - rm;
                        rm2 += (e >= sobel_lo && e <= sobel_hi) ? dv * dv : 0.f;
                    }
                    chan_merge_f(n_t, mean_t, m2_t, static_cast<float>(rc), rm, rm2);
                }
            }
#pragma unroll
            for (int e = 0; e < kLanePx; ++e) {
                h1a[e] = h1b[e]; h2a[e] = h2b[e];
                h1b[e] = h1[e]; h2b[e] = h2[e];
            }
        }
        // block reduction (fixed order, fp64) -> one partial per (frame, tile)
        int64_t cnt = static_cast<int64_t>(n_t);
        double mean = mean_t, m2 = m2_t;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t nb = __shfl_xor(cnt, o, 64);
            const double mb = __shfl_xor(mean, o, 64), qb = __shfl_xor(m2, o, 64);
            // both lanes of a pair merge (lower, upper) in the same order
            if ((lane & o) == 0) chan_merge(cnt, mean, m2, nb, mb, qb);
            else {
                int64_t n2 = nb; double mm = mb, qq = qb;
                chan_merge(n2, mm, qq, cnt, mean, m2);
                cnt = n2; mean = mm; m2 = qq;
            }
        }
        d1s = static_cast<int64_t>(wave_sum_u64(static_cast<uint64_t>(d1s)));
        d2s = wave_sum_u64(d2s);
        if (lane == 0) red[wave] = {mean, m2, cnt, d1s, d2s, 0};
        __syncthreads();
        if (threadIdx.x == 0) {
            SitiPartial o = red[0];
            for (int w = 1; w < 4; ++w) {
                chan_merge(o.n, o.mean, o.m2, red[w].n, red[w].mean, red[w].m2);
                o.d1 += red[w].d1; o.d2 += red[w].d2;
            }
            part[(int64_t)f * tiles_x * bands + tile] = o;
        }
        __syncthreads();
    }
}

__global__ void siti_finalize(const SitiPartial *part, int nframes, int ntiles, int W, int H, int has_prev,
                              double *si, double *ti) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nframes) return;
    double mean = 0.0, m2 = 0.0;
    int64_t n = 0, d1 = 0;
    uint64_t d2 = 0;
    for (int t = 0; t < ntiles; ++t) {
        const SitiPartial &p = part[(int64_t)f * ntiles + t];
        chan_merge(n, mean, m2, p.n, p.mean, p.m2);
        d1 += p.d1; d2 += p.d2;
    }
    si[f] = n ? sqrt(m2 / static_cast<double>(n)) : 0.0;
    if (f == 0 && !has_prev) {
        ti[f] = __builtin_nan("");
    } else {
        const int64_t np = static_cast<int64_t>(W) * H;
        const __int128 num = static_cast<__int128>(np) * static_cast<__int128>(d2) -
                             static_cast<__int128>(d1) * static_cast<__int128>(d1);
        ti[f] = sqrt(static_cast<double>(num)) / static_cast<double>(np);
    }
}

}  // namespace pp

using namespace pp;

extern "C" int pp_siti(pp_ctx *ctx, int bitdepth, int w, int h, const void *luma, int64_t linesize,
                       int64_t frame_stride, int nframes, const void *prev, double *si, double *ti, void *stream) {
    if (!ctx || !luma || !si || !ti || nframes < 0) PP_FAIL(PP_ERR_INVALID, "null argument");
    if (bitdepth != 8 && bitdepth != 10) PP_FAIL(PP_ERR_INVALID, "bit depth %d (8 or 10)", bitdepth);
    if (w < 3 || h < 3) PP_FAIL(PP_ERR_INVALID, "frame %dx%d too small for Sobel", w, h);
    if (nframes == 0) return PP_OK;
    hipStream_t st = static_cast<hipStream_t>(stream);
    PP_HIP(hipSetDevice(ctx->device));
    const int bytes = bitdepth > 8 ? 2 : 1;
    const int tiles_x = (w + kSpan - 1) / kSpan, bands = (h + kBand - 1) / kBand;
    const int ntiles = tiles_x * bands;
    // ~4 workgroups per CU, frames chunked per workgroup (each chunk re-reads one
    // previous frame band for TI, so chunks stay long)
    int chunks = (1024 + ntiles - 1) / ntiles;
    if (chunks > nframes) chunks = nframes;
    if (chunks > 65535) chunks = 65535;
    const int chunk = (nframes + chunks - 1) / chunks;
    chunks = (nframes + chunk - 1) / chunk;
    const int a = bytes == 2 ? 16 : 8;
    const int vec = ((uintptr_t)luma % a == 0) && (linesize % a == 0) && (nframes < 2 || frame_stride % a == 0) &&
                    (!prev || (uintptr_t)prev % a == 0);
    SitiPartial *part = nullptr;
    PP_HIP(hipMallocAsync((void **)&part, sizeof(SitiPartial) * (size_t)ntiles * nframes, st));
    dim3 grid(ntiles, chunks);
    if (bytes == 2)
        hipLaunchKernelGGL(siti_kernel<uint16_t>, grid, dim3(256), 0, st, (const uint8_t *)luma, linesize,
                           frame_stride, nframes, (const uint8_t *)prev, w, h, tiles_x, bands, chunk, vec, part);
    else
        hipLaunchKernelGGL(siti_kernel<uint8_t>, grid, dim3(256), 0, st, (const uint8_t *)luma, linesize,
                           frame_stride, nframes, (const uint8_t *)prev, w, h, tiles_x, bands, chunk, vec, part);
    hipLaunchKernelGGL(siti_finalize, dim3((nframes + 255) / 256), dim3(256), 0, st, part, nframes, ntiles, w, h,
                       prev != nullptr, si, ti);
    PP_HIP(hipGetLastError());
    PP_HIP(hipFreeAsync(part, st));
    return PP_OK;
}
