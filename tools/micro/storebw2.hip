// Store-pattern microbenchmark for the STRIDED strip layout (measurement
// only): 1200 x 1080p 16-bit frames (4.98 GB) written as strips of SB bytes
// per row, one 4-wave workgroup per (frame, strip, 540-row segment), wave w
// writing rows y0 + w, y0 + w + 4, ...; 8 B per lane (the strip kernel's V
// pass).  dup: lanes past the strip store the strip's last 8 B again (the
// clamped V pass) instead of idling.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void strips(uint8_t *d, int RB, int H, int SB, int SEG, int tpf, int dup) {
    int b = blockIdx.x;
    {  // XCD-contiguous ranges, as xcd_remap
        const int n = gridDim.x, per = n / 8, rem = n % 8, k = b % 8, q = b / 8;
        b = k < rem ? k * (per + 1) + q : rem * (per + 1) + (k - rem) * per + q;
    }
    const int frame = b / tpf, t = b % tpf;
    const int nstrips = (RB + SB - 1) / SB;
    const int seg = t / nstrips, sx = t % nstrips;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int w = min(SB, RB - sx * SB);
    int x = sx * SB + lane * 8;
    const bool on = lane * 8 < w;
    if (!on && dup) x = sx * SB + w - 8;
    uint8_t *f = d + (size_t)frame * RB * H;
    const int y0 = seg * SEG, y1 = min(H, y0 + SEG);
    for (int y = y0 + wave; y < y1; y += 4) {
        if (on || dup) *reinterpret_cast<uint2 *>(f + (size_t)y * RB + x) = make_uint2(y, x);
    }
}

int main() {
    const int RB = 3840, H = 1080, F = 1200;
    const size_t bytes = (size_t)RB * H * F;
    uint8_t *d;
    (void)hipMalloc(&d, bytes);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int rep = 0; rep < 2; ++rep)
    for (int SB : {512, 480}) for (int SEG : {540, 270, 135, 64, 32, 16}) for (int dup : {0}) {
        const int nstrips = (RB + SB - 1) / SB, nseg = (H + SEG - 1) / SEG, tpf = nstrips * nseg;
        auto launch = [&] { strips<<<tpf * F, 256>>>(d, RB, H, SB, SEG, tpf, dup); };
        for (int i = 0; i < 2; ++i) launch();
        (void)hipEventRecord(a);
        for (int i = 0; i < 5; ++i) launch();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        ms /= 5;
        printf("SB=%d SEG=%d dup=%d  %.3f ms  %.1f GB/s\n", SB, SEG, dup, ms, bytes / ms / 1e6);
    }
    return 0;
}
