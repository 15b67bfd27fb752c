/*
 * oracle/spinner_oracle.c -- CPU restatement of the stall-frame compositing spec
 * "PP-STALL-1" (see DESIGN.md).   *** TEST INFRASTRUCTURE ONLY. ***
 *
 * The reference delegates stalling to the external tool bufferer==0.22.1
 * (requirements.txt:4), invoked at p03_generateAvPvs.py:236-243 with
 * "-s util/spinner-128-white.png --black-frame --force-framerate".  Its source
 * is absent and it cannot be fetched, so its compositing
 * is PARITY UNPINNED.  This repo defines the spec below and pins it with its own
 * fixtures:
 *   1. spinner RGBA8 -> Y'CbCr BT.601 limited range with libavutil/colorspace.h
 *      RGB_TO_{Y,U,V}_CCIR (10-bit fixed point); chroma of a 2x2 (4:2:0) or 2x1
 *      (4:2:2) block is computed from the summed RGB with the macros' shift
 *      argument, its alpha is (sum + n/2) >> shift;
 *   2. 10-bit formats: Y/U/V << 2, alpha stays 8-bit;
 *   3. out = (F * (255 - A) + S * A + 127) / 255 (exact integer division);
 *   4. the spinner is centred: x = (W - ws) / 2, y = (H - hs) / 2, both rounded
 *      down to the chroma grid.
 */
#include <stdint.h>
#include <string.h>

#define SCALEBITS 10
#define ONE_HALF (1 << (SCALEBITS - 1))
#define FIX(x) ((int)((x) * (1 << SCALEBITS) + 0.5))

static int rgb_to_y(int r, int g, int b)
{
    return (FIX(0.29900 * 219.0 / 255.0) * r + FIX(0.58700 * 219.0 / 255.0) * g +
            FIX(0.11400 * 219.0 / 255.0) * b + (ONE_HALF + (16 << SCALEBITS))) >> SCALEBITS;
}
static int rgb_to_u(int r1, int g1, int b1, int shift)
{
    return ((-FIX(0.16874 * 224.0 / 255.0) * r1 - FIX(0.33126 * 224.0 / 255.0) * g1 +
             FIX(0.50000 * 224.0 / 255.0) * b1 + (ONE_HALF << shift) - 1) >> (SCALEBITS + shift)) + 128;
}
static int rgb_to_v(int r1, int g1, int b1, int shift)
{
    return ((FIX(0.50000 * 224.0 / 255.0) * r1 - FIX(0.41869 * 224.0 / 255.0) * g1 -
             FIX(0.08131 * 224.0 / 255.0) * b1 + (ONE_HALF << shift) - 1) >> (SCALEBITS + shift)) + 128;
}

/*
 * rgba: w*h*4 bytes.  Outputs (all uint16, code values at `depth`):
 *   Y[w*h], A_l[w*h] (8-bit alpha), U/V/A_c[cw*ch] with cw = w >> hsub, ch = h >> vsub.
 * w and h must be multiples of the chroma block.
 */
int po_spinner_to_yuva(const uint8_t *rgba, int w, int h, int hsub, int vsub, int depth,
                       uint16_t *Y, uint16_t *Al, uint16_t *U, uint16_t *V, uint16_t *Ac)
{
    int cw = w >> hsub, ch = h >> vsub, sh = depth - 8, shift = hsub + vsub;
    if ((w & ((1 << hsub) - 1)) || (h & ((1 << vsub) - 1))) return -1;
    for (int i = 0; i < w * h; i++) {
        const uint8_t *p = rgba + 4 * i;
        Y[i] = (uint16_t)(rgb_to_y(p[0], p[1], p[2]) << sh);
        Al[i] = p[3];
    }
    for (int cy = 0; cy < ch; cy++)
        for (int cx = 0; cx < cw; cx++) {
            int r = 0, g = 0, b = 0, a = 0;
            for (int dy = 0; dy < (1 << vsub); dy++)
                for (int dx = 0; dx < (1 << hsub); dx++) {
                    const uint8_t *p = rgba + 4 * ((size_t)((cy << vsub) + dy) * w + (cx << hsub) + dx);
                    r += p[0]; g += p[1]; b += p[2]; a += p[3];
                }
            U[cy * cw + cx] = (uint16_t)(rgb_to_u(r, g, b, shift) << sh);
            V[cy * cw + cx] = (uint16_t)(rgb_to_v(r, g, b, shift) << sh);
            Ac[cy * cw + cx] = (uint16_t)((a + ((1 << shift) >> 1)) >> shift);
        }
    return 0;
}

/* Blend one spinner plane (S, A: sw x sh, uint16) into plane D at (ox, oy). */
static void blend_plane(uint8_t *D, int64_t ls, int bps, const uint16_t *S, const uint16_t *A,
                        int sw, int sh, int ox, int oy, int W, int H)
{
    for (int y = 0; y < sh; y++) {
        int yy = oy + y;
        if (yy < 0 || yy >= H) continue;
        uint8_t *row = D + (int64_t)yy * ls;
        for (int x = 0; x < sw; x++) {
            int xx = ox + x, f, a = A[y * sw + x], s = S[y * sw + x];
            if (xx < 0 || xx >= W) continue;
            f = bps == 1 ? row[xx] : ((uint16_t *)row)[xx];
            f = (f * (255 - a) + s * a + 127) / 255;
            if (bps == 1) row[xx] = (uint8_t)f; else ((uint16_t *)row)[xx] = (uint16_t)f;
        }
    }
}

/* Composite in place.  planes/ls: frame planes; W x H luma; spinner prepared by
 * po_spinner_to_yuva for the same hsub/vsub/depth. */
int po_overlay_spinner(uint8_t *const planes[3], const int64_t ls[3], int W, int H, int hsub, int vsub,
                       int depth, const uint16_t *Y, const uint16_t *Al, const uint16_t *U,
                       const uint16_t *V, const uint16_t *Ac, int sw, int sh)
{
    int bps = depth > 8 ? 2 : 1;
    int x0 = ((W - sw) / 2) >> hsub << hsub, y0 = ((H - sh) / 2) >> vsub << vsub;
    int cw = sw >> hsub, ch = sh >> vsub;
    int CW = -((-W) >> hsub), CH = -((-H) >> vsub);
    blend_plane(planes[0], ls[0], bps, Y, Al, sw, sh, x0, y0, W, H);
    blend_plane(planes[1], ls[1], bps, U, Ac, cw, ch, x0 >> hsub, y0 >> vsub, CW, CH);
    blend_plane(planes[2], ls[2], bps, V, Ac, cw, ch, x0 >> hsub, y0 >> vsub, CW, CH);
    return 0;
}
