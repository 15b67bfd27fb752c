// Store-bandwidth microbenchmark (measurement only): how fast can gfx950 write
// 5 GB of frame data with the strip kernel's store shapes?
//   mode 0: dwordx4 per lane, fully contiguous (streaming memset)
//   mode 1: dwordx2 per lane, fully contiguous
//   mode 2: dwordx2, 512-B row segments of 3840-B rows (the strip kernel's luma pattern:
//           workgroup = one 256-column strip, rows walked top to bottom)
//   mode 3: dwordx4, 1024-B segments (512 columns per workgroup)
//   mode 4: dwordx4, whole 3840-B rows per workgroup (row-major walk)
//   mode 5: copy (read 1 B : write 1 B, dwordx4) for reference
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256) void contig4(uint4 *d, size_t n) {
    size_t i = blockIdx.x * 256ull + threadIdx.x;
    const size_t step = (size_t)gridDim.x * 256;
    for (; i < n; i += step) d[i] = make_uint4((uint32_t)i, 1, 2, 3);
}
__global__ __launch_bounds__(256) void contig2(uint2 *d, size_t n) {
    size_t i = blockIdx.x * 256ull + threadIdx.x;
    const size_t step = (size_t)gridDim.x * 256;
    for (; i < n; i += step) d[i] = make_uint2((uint32_t)i, 1);
}
// frames of H rows x RB bytes; workgroup = (frame, strip of SB bytes, segment of SEG rows); 4 waves take rows y+wave
template <int W>  // bytes per lane store: 8 or 16
__global__ __launch_bounds__(256) void strips(uint8_t *d, int RB, int H, int SB, int SEG, int tiles_per_frame) {
    const int b = blockIdx.x;
    const int frame = b / tiles_per_frame, t = b % tiles_per_frame;
    const int nstrips = (RB + SB - 1) / SB;
    const int seg = t / nstrips, sx = t % nstrips;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int x = sx * SB + lane * W;
    uint8_t *f = d + (size_t)frame * RB * H;
    const int y0 = seg * SEG, y1 = min(H, y0 + SEG);
    for (int y = y0 + wave; y < y1; y += 4) {
        for (int xx = x; xx < min(RB, sx * SB + SB); xx += 64 * W) {
            if constexpr (W == 16) *reinterpret_cast<uint4 *>(f + (size_t)y * RB + xx) = make_uint4(y, xx, 0, 1);
            else *reinterpret_cast<uint2 *>(f + (size_t)y * RB + xx) = make_uint2(y, xx);
        }
    }
}
__global__ __launch_bounds__(256) void copy4(const uint4 *s, uint4 *d, size_t n) {
    size_t i = blockIdx.x * 256ull + threadIdx.x;
    const size_t step = (size_t)gridDim.x * 256;
    for (; i < n; i += step) d[i] = s[i];
}

int main() {
    const int RB = 3840, H = 1080, F = 1200;  // 1200 luma frames of 1080p 16-bit = 4.98 GB
    const size_t bytes = (size_t)RB * H * F;
    uint8_t *d, *s;
    hipMalloc(&d, bytes);
    hipMalloc(&s, bytes / 2);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](const char *name, auto launch, double nbytes) {
        for (int i = 0; i < 2; ++i) launch();
        hipEventRecord(a);
        const int R = 5;
        for (int i = 0; i < R; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        ms /= R;
        printf("%-44s %8.3f ms  %7.1f GB/s\n", name, ms, nbytes / ms / 1e6);
    };
    run("contig dwordx4 (grid 256x16 persistent)", [&] { contig4<<<4096, 256>>>((uint4 *)d, bytes / 16); }, bytes);
    run("contig dwordx4 (grid = n/256)", [&] { contig4<<<(unsigned)(bytes / 16 / 256), 256>>>((uint4 *)d, bytes / 16); }, bytes);
    run("contig dwordx2 (grid 4096)", [&] { contig2<<<4096, 256>>>((uint2 *)d, bytes / 8); }, bytes);
    for (int SB : {512, 1024, 3840}) {
        for (int SEG : {270, 1080}) {
            const int nstrips = (RB + SB - 1) / SB, nseg = (H + SEG - 1) / SEG;
            const int tpf = nstrips * nseg;
            char nm[96];
            snprintf(nm, sizeof nm, "strips x2  SB=%d SEG=%d", SB, SEG);
            run(nm, [&] { strips<8><<<tpf * F, 256>>>(d, RB, H, SB, SEG, tpf); }, bytes);
            snprintf(nm, sizeof nm, "strips x4  SB=%d SEG=%d", SB, SEG);
            run(nm, [&] { strips<16><<<tpf * F, 256>>>(d, RB, H, SB, SEG, tpf); }, bytes);
        }
    }
    run("copy dwordx4 (2.49 GB read + write)", [&] { copy4<<<4096, 256>>>((const uint4 *)s, (uint4 *)d, bytes / 32); }, bytes);
    run("hipMemsetAsync", [&] { hipMemsetAsync(d, 1, bytes); }, bytes);
    hipFree(d);
    hipFree(s);
    return 0;
}
