// Host-side polyphase filter-bank construction for the scaler plans.
//
// Restates FFmpeg 7.0 libswscale/utils.c initFilter() (the reference pins
// FFmpeg 7.0.2, docker/install_ffmpeg.sh:39-41; call sites lib/ffmpeg.py:800,
// :992, :1038, :1213) for the three filters the reference can request
// (flags=bicubic at every call site; lanczos and bilinear for the north_star
// configs) with the x86 build's alignment (filterAlign H=4, V=2), no
// SWS_BITEXACT, no user src/dst vectors.  The result is the exact int16 table
// FFmpeg feeds its hScale/yuv2planeX loops; `compact()` then re-windows it for
// the GPU without changing any product.
#include "filters.hpp"

#include <cmath>
#include <cstdlib>

namespace pp {

namespace {

constexpr double kParamDefault = 123456.0;  // SWS_PARAM_DEFAULT
constexpr double kReduceCutoff = 0.002;     // SWS_MAX_REDUCE_CUTOFF
constexpr int kMaxTaps = 64;

int ilog2(unsigned v) {
    int n = 0;
    while (v > 1) { v >>= 1; ++n; }
    return n;
}

// Kernel value for one tap at distance d (2^30 = one source sample), in units of fone.
int64_t tap_weight(int flags, int64_t d, int64_t fone, double p0, double p1) {
    const double fd = static_cast<double>(d) * (1.0 / (1 << 30));
    if (flags & PP_SWS_BICUBIC) {
        const int64_t B = static_cast<int64_t>((p0 != kParamDefault ? p0 : 0.0) * (1 << 24));
        const int64_t C = static_cast<int64_t>((p1 != kParamDefault ? p1 : 0.6) * (1 << 24));
        int64_t w = 0;
        if (d < (int64_t(1) << 31)) {
            const int64_t d2 = (d * d) >> 30;
            const int64_t d3 = (d2 * d) >> 30;
            if (d < (int64_t(1) << 30))
                w = (12 * (1 << 24) - 9 * B - 6 * C) * d3 + (-18 * (1 << 24) + 12 * B + 6 * C) * d2 +
                    (6 * (1 << 24) - 2 * B) * (int64_t(1) << 30);
            else
                w = (-B - 6 * C) * d3 + (6 * B + 30 * C) * d2 + (-12 * B - 48 * C) * d +
                    (8 * B + 24 * C) * (int64_t(1) << 30);
        }
        return w / ((int64_t(1) << 54) / fone);
    }
    if (flags & PP_SWS_LANCZOS) {
        const double p = p0 != kParamDefault ? p0 : 3.0;
        int64_t w = static_cast<int64_t>(
            (d ? std::sin(fd * M_PI) * std::sin(fd * M_PI / p) / (fd * fd * M_PI * M_PI / p) : 1.0) * fone);
        return fd > p ? 0 : w;
    }
    // bilinear
    int64_t w = (int64_t(1) << 30) - d;
    return (w < 0 ? 0 : w) * (fone >> 30);
}

}  // namespace

int FilterBank::build(int xinc, int src_n, int dst_n, int align, int one, int flags, double p0,
                      double p1, int src_pos, int dst_pos, std::string *err) {
    n = dst_n;
    const int ratio_log = ilog2(static_cast<unsigned>(src_n / dst_n));
    const int64_t fone = int64_t(1) << (54 - (ratio_log < 8 ? ratio_log : 8));

    // 1. raw taps (width `w`) and window starts
    int w;
    std::vector<int64_t> raw;
    pos.assign(dst_n, 0);
    if (std::abs(xinc - 0x10000) < 10 && src_pos == dst_pos) {
        w = 1;
        raw.assign(dst_n, fone);
        for (int i = 0; i < dst_n; ++i) pos[i] = i;
    } else {
        int size_factor;
        if (flags & PP_SWS_LANCZOS)
            size_factor = p0 != kParamDefault ? static_cast<int>(std::ceil(2 * p0)) : 6;
        else if (flags & PP_SWS_BICUBIC)
            size_factor = 4;
        else if (flags & PP_SWS_BILINEAR)
            size_factor = 2;
        else {
            *err = "unsupported scaler flags";
            return -1;
        }
        w = xinc <= (1 << 16) ? 1 + size_factor : 1 + (size_factor * src_n + dst_n - 1) / dst_n;
        if (w > src_n - 2) w = src_n - 2;
        if (w < 1) w = 1;
        if (w > kMaxTaps) {
            *err = "filter too long (scale ratio too large)";
            return -1;
        }
        raw.assign(static_cast<size_t>(dst_n) * w, 0);
        int64_t center = ((dst_pos * int64_t(xinc)) >> 7) - ((src_pos * int64_t(0x10000)) >> 7);
        for (int i = 0; i < dst_n; ++i, center += 2 * int64_t(xinc)) {
            // C integer division truncates toward zero; FFmpeg relies on it.
            int first = static_cast<int>((center - (w - 2) * (int64_t(1) << 16)) / (1 << 17));
            pos[i] = first;
            for (int j = 0; j < w; ++j) {
                int64_t d = std::llabs(int64_t(first + j) * (1 << 17) - center) << 13;
                if (xinc > (1 << 16)) d = d * dst_n / src_n;
                raw[static_cast<size_t>(i) * w + j] = tap_weight(flags, d, fone, p0, p1);
            }
        }
    }

    // 2. shrink: drop near-zero taps on the left (moving the window), count them on the right
    int needed = 0;
    for (int i = dst_n - 1; i >= 0; --i) {
        int64_t *f = &raw[static_cast<size_t>(i) * w];
        int64_t acc = 0;
        for (int j = 0; j < w; ++j) {
            acc += std::llabs(f[0]);
            if (acc > kReduceCutoff * fone) break;
            if (i < dst_n - 1 && pos[i] >= pos[i + 1]) break;
            for (int k = 1; k < w; ++k) f[k - 1] = f[k];
            f[w - 1] = 0;
            ++pos[i];
        }
        int keep = w;
        acc = 0;
        for (int j = w - 1; j > 0; --j) {
            acc += std::llabs(f[j]);
            if (acc > kReduceCutoff * fone) break;
            --keep;
        }
        if (keep > needed) needed = keep;
    }
    if (needed == 1 && align == 2) align = 1;  // x86 MMX unscaled-vertical special case
    size = (needed + align - 1) & ~(align - 1);
    if (size > kMaxTaps) {
        *err = "filter too long after alignment";
        return -1;
    }
    std::vector<int64_t> f(static_cast<size_t>(dst_n) * size, 0);
    for (int i = 0; i < dst_n; ++i)
        for (int j = 0; j < size && j < w; ++j) f[static_cast<size_t>(i) * size + j] = raw[static_cast<size_t>(i) * w + j];

    // 3. fold taps that fall outside [0, src_n) onto the edge samples
    for (int i = 0; i < dst_n; ++i) {
        int64_t *c = &f[static_cast<size_t>(i) * size];
        if (pos[i] < 0) {
            for (int j = 1; j < size; ++j) {
                const int left = j + pos[i] > 0 ? j + pos[i] : 0;
                c[left] += c[j];
                c[j] = 0;
            }
            pos[i] = 0;
        }
        if (pos[i] + size > src_n) {
            const int shift = pos[i] + (size - src_n < 0 ? size - src_n : 0);
            int64_t over = 0;
            for (int j = size - 1; j >= 0; --j)
                if (pos[i] + j >= src_n) {
                    over += c[j];
                    c[j] = 0;
                }
            for (int j = size - 1; j >= 0; --j) c[j] = j < shift ? 0 : c[j - shift];
            pos[i] -= shift;
            c[src_n - 1 - pos[i]] += over;
        }
    }

    // 4. normalise to `one` with error diffusion (ROUNDED_DIV)
    coef.assign(static_cast<size_t>(dst_n) * size, 0);
    for (int i = 0; i < dst_n; ++i) {
        const int64_t *c = &f[static_cast<size_t>(i) * size];
        int64_t sum = 0;
        for (int j = 0; j < size; ++j) sum += c[j];
        sum = (sum + one / 2) / one;
        if (!sum) sum = 1;
        int64_t carry = 0;
        for (int j = 0; j < size; ++j) {
            const int64_t v = c[j] + carry;
            const int64_t q = (v >= 0 ? v + (sum >> 1) : v - (sum >> 1)) / sum;
            coef[static_cast<size_t>(i) * size + j] = static_cast<int16_t>(q);
            carry = v - q * sum;
        }
    }
    return 0;
}

int FilterBank::compact(int src_n, int bucket_min, Compact *out, std::string *err) const {
    // Narrowest window holding every non-zero tap of every output.
    int span = 1;
    std::vector<int> lo(n, 0);
    for (int i = 0; i < n; ++i) {
        const int16_t *c = &coef[static_cast<size_t>(i) * size];
        int a = 0, b = 0;
        bool any = false;
        for (int j = 0; j < size; ++j)
            if (c[j]) {
                if (!any) a = j;
                b = j;
                any = true;
            }
        lo[i] = any ? a : 0;
        if (any && b - a + 1 > span) span = b - a + 1;
    }
    int taps = span;
    if (taps < bucket_min) taps = bucket_min;
    if (span > src_n) {
        *err = "source plane narrower than the filter";
        return -1;
    }
    // a window wider than the plane (tiny planes, bucketed taps) starts at 0; the
    // kernel's staging zero-fills samples past the plane edge
    out->taps = taps;
    out->pos.assign(n, 0);
    out->coef.assign(static_cast<size_t>(n) * taps, 0);
    for (int i = 0; i < n; ++i) {
        int start = pos[i] + lo[i];
        if (start + taps > src_n) start = src_n - taps;  // window slides left, leading zeros
        if (start < 0) start = 0;
        out->pos[i] = start;
        const int16_t *c = &coef[static_cast<size_t>(i) * size];
        for (int j = 0; j < size; ++j) {
            if (!c[j]) continue;
            const int k = pos[i] + j - start;
            if (k < 0 || k >= taps) {
                *err = "internal: compaction window";
                return -1;
            }
            out->coef[static_cast<size_t>(i) * taps + k] = c[j];
        }
    }
    return 0;
}

}  // namespace pp
