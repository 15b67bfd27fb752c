// V-pass store microbenchmark (measurement only): 1200 x 1080p 16-bit frames
// (4.98 GB) written in the strip kernel's shape -- a 4-wave workgroup owns a
// 512-B wide strip x SEG rows, wave w writes rows y0+w, y0+w+4, ... -- with K
// dependent VALU ops per row before its store, and the workgroups per CU
// limited by dynamic LDS.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v2s __attribute__((ext_vector_type(2)));

template <int W, int K>
__global__ __launch_bounds__(256) void vstore(uint8_t *d, int RB, int H, int SB, int SEG, int tpf, int remap) {
    extern __shared__ int lds[];
    int b = blockIdx.x;
    if (remap) {  // XCD-contiguous ranges, as xcd_remap
        const int n = gridDim.x, per = n / 8, rem = n % 8, k = b % 8, q = b / 8;
        b = k < rem ? k * (per + 1) + q : rem * (per + 1) + (k - rem) * per + q;
    }
    const int frame = b / tpf, t = b % tpf;
    const int nstrips = (RB + SB - 1) / SB;
    const int seg = t / nstrips, sx = t % nstrips;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int x = sx * SB + lane * W;
    uint8_t *f = d + (size_t)frame * RB * H;
    const int y0 = seg * SEG, y1 = min(H, y0 + SEG);
    uint32_t acc = lane * 2654435761u;
    if (threadIdx.x == 0) lds[0] = 0;
    for (int y = y0 + wave; y < y1; y += 4) {
#pragma unroll
        for (int k = 0; k < K; ++k) acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2s, acc), v2s{3, 5}, (int)acc, false);
        if (x < min(RB, sx * SB + SB)) {
            if constexpr (W == 16) *reinterpret_cast<uint4 *>(f + (size_t)y * RB + x) = make_uint4(acc, y, acc, 1);
            else *reinterpret_cast<uint2 *>(f + (size_t)y * RB + x) = make_uint2(acc, y);
        }
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
    auto run = [&](const char *name, auto launch) {
        for (int i = 0; i < 2; ++i) launch();
        (void)hipEventRecord(a);
        for (int i = 0; i < 5; ++i) launch();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        ms /= 5;
        printf("%-56s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6);
    };
    const int SEG = 270, SB = 512;
    const int tpf = ((RB + SB - 1) / SB) * ((H + SEG - 1) / SEG);
    const unsigned grid = tpf * F;
    for (int ldskb : {0, 20, 26, 40}) {
        for (int remap : {0, 1}) {
            char nm[128];
#define RUN(WW, KK)                                                                                      \
    snprintf(nm, sizeof nm, "W=%d K=%d lds=%dKB remap=%d", WW, KK, ldskb, remap);                        \
    run(nm, [&] { vstore<WW, KK><<<grid, 256, ldskb * 1024>>>(d, RB, H, SB, SEG, tpf, remap); });
            RUN(8, 0) RUN(8, 24) RUN(8, 48)
            if (remap == 0) { RUN(16, 0) RUN(16, 48) }
        }
    }
    (void)hipFree(d);
    return 0;
}
