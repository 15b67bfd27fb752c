/*
 * oracle/siti_oracle.c -- CPU restatement of ITU-T P.910 SI/TI (spec "PP-SITI-1").
 *
 *   *** TEST INFRASTRUCTURE ONLY (checker + cpu_baseline). ***
 *
 * The reference has no SI/TI code: util/SRC_analysis.py
 * (analyse_src, :120-147) and util/complexity_classification.py
 * (get_difficulty, :50-69) are the designated hooks (BASELINE.json north_star).
 * The spec this file and oracle/siti_ref.py (numpy) implement, and the product
 * kernel must match within 1e-4 relative:
 *   - luma plane only, raw code values at native bit depth (8: uint8, 10: uint16 LE);
 *   - Sobel 3x3, Gx = [[-1,0,1],[-2,0,2],[-1,0,1]], Gy = Gx^T, evaluated on the
 *     "valid" region (rows 1..H-2, cols 1..W-2; the 1-px border is dropped);
 *   - SI_n = population std (ddof = 0) of sqrt(Gx^2 + Gy^2) over that region;
 *   - TI_n = population std of Y_n - Y_{n-1} over the full frame, n >= 1
 *     (TI_0 is undefined and reported as NaN);
 *   - SI = max_n SI_n, TI = max_n TI_n.
 * PARITY STATUS: parity unpinned against the reference (no implementation
 * exists); pinned by the known-answer tests in tests/test_oracle_siti.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

static inline int px(const uint8_t *base, int64_t ls, int bd, int x, int y)
{
    const uint8_t *row = base + (int64_t)y * ls;
    return bd == 8 ? row[x] : ((const uint16_t *)row)[x];
}

/* Two-pass (mean, then squared deviations) in double, like numpy.std. */
double po_si_frame(const uint8_t *Y, int64_t ls, int w, int h, int bd)
{
    int64_t n = (int64_t)(w - 2) * (h - 2);
    double *m;
    double sum = 0, var = 0, mean;
    if (w < 3 || h < 3) return NAN;
    m = malloc((size_t)n * sizeof(double));
    if (!m) return NAN;
    int64_t k = 0;
    for (int y = 1; y < h - 1; y++) {
        for (int x = 1; x < w - 1; x++) {
            int a0 = px(Y, ls, bd, x - 1, y - 1), a1 = px(Y, ls, bd, x, y - 1), a2 = px(Y, ls, bd, x + 1, y - 1);
            int b0 = px(Y, ls, bd, x - 1, y), b2 = px(Y, ls, bd, x + 1, y);
            int c0 = px(Y, ls, bd, x - 1, y + 1), c1 = px(Y, ls, bd, x, y + 1), c2 = px(Y, ls, bd, x + 1, y + 1);
            int gx = (a2 - a0) + 2 * (b2 - b0) + (c2 - c0);
            int gy = (c0 + 2 * c1 + c2) - (a0 + 2 * a1 + a2);
            double g = sqrt((double)gx * gx + (double)gy * gy);
            m[k++] = g;
            sum += g;
        }
    }
    mean = sum / (double)n;
    for (k = 0; k < n; k++) {
        double d = m[k] - mean;
        var += d * d;
    }
    free(m);
    return sqrt(var / (double)n);
}

double po_ti_frame(const uint8_t *Y, const uint8_t *P, int64_t ls, int w, int h, int bd)
{
    int64_t n = (int64_t)w * h;
    int64_t s1 = 0, s2 = 0;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            int64_t d = px(Y, ls, bd, x, y) - px(P, ls, bd, x, y);
            s1 += d;
            s2 += d * d;
        }
    /* exact integer moments: var = (n*s2 - s1^2) / n^2, numerator in 128 bit */
    {
        __int128 num = (__int128)n * s2 - (__int128)s1 * s1;
        return sqrt((double)num) / (double)n;
    }
}

/* Per-frame SI/TI over a contiguous batch; prev (may be NULL) is frame -1. */
void po_siti_batch(const uint8_t *frames, int64_t ls, int64_t fstride, int nframes, int w, int h,
                   int bd, const uint8_t *prev, double *si, double *ti)
{
    for (int f = 0; f < nframes; f++) {
        const uint8_t *cur = frames + (int64_t)f * fstride;
        const uint8_t *p = f ? frames + (int64_t)(f - 1) * fstride : prev;
        si[f] = po_si_frame(cur, ls, w, h, bd);
        ti[f] = p ? po_ti_frame(cur, p, ls, w, h, bd) : NAN;
    }
}
