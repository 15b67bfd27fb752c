// Traffic floor of the config-2 scaler (measurement only): each 4-wave
// workgroup reads its strip of a 1280x720 16-bit plane (16-B lanes) and writes
// its strip of the 1920x1080 plane (8-B lanes), rows in the kernel's order,
// no arithmetic.  3 planes (yuv422p10le), 600 frames = 2.2 GB read + 5.0 GB
// written, the strip kernel's algorithmic bytes.
#include <hip/hip_runtime.h>
#include <cstdio>

struct Plane { const uint8_t *s; uint8_t *d; int sw, sh, dw, dh; };

__global__ __launch_bounds__(256) void stripcopy(Plane p0, Plane p1, Plane p2, int tiles_l, int tiles_c, int SEG,
                                                 int remap, int wbytes) {
    int b = blockIdx.x;
    if (remap) {
        const int n = gridDim.x, per = n / 8, rem = n % 8, k = b % 8, q = b / 8;
        b = k < rem ? k * (per + 1) + q : rem * (per + 1) + (k - rem) * per + q;
    }
    const int tpf = tiles_l + 2 * tiles_c;
    const int frame = b / tpf;
    int t = b % tpf;
    Plane P = p0;
    int tiles = tiles_l;
    if (t >= tiles_l) { t -= tiles_l; P = p1; tiles = tiles_c; if (t >= tiles_c) { t -= tiles_c; P = p2; } }
    const int nstrips = (P.dw + 255) / 256;
    const int seg = t / nstrips, sx = t % nstrips;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint8_t *S = P.s + (size_t)frame * P.sw * P.sh * 2;
    uint8_t *D = P.d + (size_t)frame * P.dw * P.dh * 2;
    const int y0 = seg * SEG, y1 = min(P.dh, y0 + SEG);
    // source rows of this segment: ~(y1-y0)*sh/dh, strip width ~ 256*sw/dw samples
    const int sx0 = sx * 256 * P.sw / P.dw, sxw = 176;
    const int sy0 = y0 * P.sh / P.dh, sy1 = min(P.sh, (y1 * P.sh + P.dh - 1) / P.dh + 4);
    uint32_t acc = 0;
    for (int y = sy0 + (threadIdx.x / 22); y < sy1; y += 256 / 22) {
        const int c = (threadIdx.x % 22) * 8;
        if (threadIdx.x < 242 && sx0 + c + 8 <= P.sw && c < sxw) {
            const uint4 v = *reinterpret_cast<const uint4 *>(S + ((size_t)y * P.sw + sx0 + c) * 2);
            acc ^= v.x ^ v.w;
        }
    }
    const int x = sx * 256 + lane * 4;
    for (int y = y0 + wave; y < y1; y += 4) {
        if (x < P.dw) *reinterpret_cast<uint2 *>(D + ((size_t)y * P.dw + x) * 2) = make_uint2(acc + y, x);
    }
}

int main() {
    const int F = 600;
    Plane pl[3];
    int sw[3] = {1280, 640, 640}, dw[3] = {1920, 960, 960};
    for (int p = 0; p < 3; ++p) {
        pl[p].sw = sw[p]; pl[p].sh = 720; pl[p].dw = dw[p]; pl[p].dh = 1080;
        (void)hipMalloc((void **)&pl[p].s, (size_t)sw[p] * 720 * 2 * F);
        (void)hipMalloc((void **)&pl[p].d, (size_t)dw[p] * 1080 * 2 * F);
    }
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const double bytes = 600.0 * (3686400 + 8294400);
    for (int SEG : {270, 540}) for (int remap : {0, 1}) {
        const int nseg = (1080 + SEG - 1) / SEG;
        const int tl = 8 * nseg, tc = 4 * nseg;
        const unsigned grid = (tl + 2 * tc) * F;
        for (int i = 0; i < 2; ++i) stripcopy<<<grid, 256, 26 * 1024>>>(pl[0], pl[1], pl[2], tl, tc, SEG, remap, 8);
        (void)hipEventRecord(a);
        for (int i = 0; i < 5; ++i) stripcopy<<<grid, 256, 26 * 1024>>>(pl[0], pl[1], pl[2], tl, tc, SEG, remap, 8);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        ms /= 5;
        printf("stripcopy SEG=%d remap=%d  %.3f ms  %.1f GB/s (algorithmic)\n", SEG, remap, ms, bytes / ms / 1e6);
    }
    return 0;
}
