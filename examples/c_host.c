/*
 * c_host.c -- a host without torch or Python driving the pixel path through
 * the C ABI only (include/pixpath.h): pinned host batch -> H2D on a copy
 * stream -> lanczos 1280x720 -> 1920x1080 yuv422p10le (create_avpvs_short's
 * scale, lib/ffmpeg.py:992) -> v210 CPVS (create_cpvs, lib/ffmpeg.py:1198) on
 * a compute stream ordered by an event -> D2H -> file.
 *
 *   gcc -O2 -Iinclude examples/c_host.c -Lprocessing-chain_amd/pixpath -lpixpath \
 *       -Wl,-rpath,$PWD/processing-chain_amd/pixpath -o c_host
 *   ./c_host NFRAMES out.v210        (input: sample(f, p, x, y) below)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pixpath.h"

#define CHECK(x)                                                              \
    do {                                                                      \
        int rc_ = (x);                                                        \
        if (rc_ < 0) {                                                        \
            fprintf(stderr, "%s failed (%d): %s\n", #x, rc_, pp_last_error()); \
            return 1;                                                         \
        }                                                                     \
    } while (0)

enum { SW = 1280, SH = 720, DW = 1920, DH = 1080 };

/* deterministic 10-bit legal-range test pattern (the pytest recomputes it) */
static unsigned short sample(int f, int p, int x, int y) {
    unsigned v = (unsigned)(x * 7 + y * 13 + f * 29 + p * 101) ^ (unsigned)((x * y + f) * 2654435761u >> 20);
    return (unsigned short)(64 + v % 877);
}

/* a dense frame-interleaved yuv422p10le batch in one buffer */
static void dense_frames(pp_frames *fr, void *base, int w, int h) {
    const int64_t y = (int64_t)w * 2 * h, c = (int64_t)(w / 2) * 2 * h;
    fr->data[0] = base;
    fr->data[1] = (char *)base + y;
    fr->data[2] = (char *)base + y + c;
    fr->linesize[0] = (int64_t)w * 2;
    fr->linesize[1] = fr->linesize[2] = (int64_t)(w / 2) * 2;
    fr->frame_stride[0] = fr->frame_stride[1] = fr->frame_stride[2] = y + 2 * c;
}

int main(int argc, char **argv) {
    if (argc != 3) {
        fprintf(stderr, "usage: %s NFRAMES out.v210\n", argv[0]);
        return 2;
    }
    const int n = atoi(argv[1]);
    if (n < 1) return 2;
    if (pp_abi_version() != PP_ABI_VERSION) {
        fprintf(stderr, "ABI %d, header %d\n", pp_abi_version(), PP_ABI_VERSION);
        return 1;
    }
    pp_ctx *ctx = NULL;
    CHECK(pp_ctx_create(0, &ctx));
    const int64_t in_frame = (int64_t)SW * SH * 2 * 2, mid_frame = (int64_t)DW * DH * 2 * 2;
    const int64_t v210_line = pp_v210_linesize(DW), out_frame = v210_line * DH;
    void *h_in = NULL, *h_out = NULL, *d_in = NULL, *d_mid = NULL, *d_out = NULL;
    CHECK(pp_host_alloc(in_frame * n, &h_in));
    CHECK(pp_host_alloc(out_frame * n, &h_out));
    CHECK(pp_device_alloc(ctx, in_frame * n, &d_in));
    CHECK(pp_device_alloc(ctx, mid_frame * n, &d_mid));
    CHECK(pp_device_alloc(ctx, out_frame * n, &d_out));
    pp_frames hin, din, dmid, dout, hout;
    dense_frames(&hin, h_in, SW, SH);
    dense_frames(&din, d_in, SW, SH);
    dense_frames(&dmid, d_mid, DW, DH);
    for (int f = 0; f < n; ++f)
        for (int p = 0; p < 3; ++p) {
            unsigned short *pl = (unsigned short *)((char *)hin.data[p] + f * hin.frame_stride[p]);
            const int pw = p ? SW / 2 : SW;
            for (int y = 0; y < SH; ++y)
                for (int x = 0; x < pw; ++x) pl[(int64_t)y * pw + x] = sample(f, p, x, y);
        }
    memset(&dout, 0, sizeof dout);
    dout.data[0] = d_out;
    dout.linesize[0] = v210_line;
    dout.frame_stride[0] = out_frame;
    hout = dout;
    hout.data[0] = h_out;

    void *copy = NULL, *compute = NULL, *uploaded = NULL, *done = NULL, *t0 = NULL;
    CHECK(pp_stream_create(ctx, &copy));
    CHECK(pp_stream_create(ctx, &compute));
    CHECK(pp_event_create(ctx, &uploaded));
    CHECK(pp_event_create(ctx, &done));
    CHECK(pp_event_create(ctx, &t0));
    pp_scale_plan *plan = NULL;
    CHECK(pp_scale_plan_create(ctx, PP_FMT_YUV422P10LE, SW, SH, PP_FMT_YUV422P10LE, DW, DH, PP_SWS_LANCZOS,
                               PP_SWS_PARAM_DEFAULT, PP_SWS_PARAM_DEFAULT, &plan));

    CHECK(pp_frames_copy_async(PP_FMT_YUV422P10LE, SW, SH, &din, &hin, n, PP_COPY_H2D, copy));
    CHECK(pp_event_record(uploaded, copy));
    CHECK(pp_stream_wait_event(compute, uploaded));
    CHECK(pp_event_record(t0, compute));
    CHECK(pp_scale_execute(plan, &din, &dmid, n, compute));
    CHECK(pp_cpvs_execute(ctx, PP_FMT_YUV422P10LE, DW, DH, &dmid, DW, DH, -1, -1, PP_FMT_V210, &dout, n, compute));
    CHECK(pp_event_record(done, compute));
    CHECK(pp_stream_wait_event(copy, done));
    CHECK(pp_frames_copy_async(PP_FMT_V210, DW, DH, &hout, &dout, n, PP_COPY_D2H, copy));
    CHECK(pp_stream_synchronize(copy));
    float ms = 0.f;
    CHECK(pp_event_elapsed_ms(t0, done, &ms));

    FILE *fo = fopen(argv[2], "wb");
    if (!fo || fwrite(h_out, 1, (size_t)(out_frame * n), fo) != (size_t)(out_frame * n)) {
        fprintf(stderr, "cannot write %s\n", argv[2]);
        return 1;
    }
    fclose(fo);
    printf("frames %d kernels_ms %.4f\n", n, ms);

    CHECK(pp_scale_plan_destroy(plan));
    CHECK(pp_event_destroy(t0));
    CHECK(pp_event_destroy(done));
    CHECK(pp_event_destroy(uploaded));
    CHECK(pp_stream_destroy(ctx, compute));
    CHECK(pp_stream_destroy(ctx, copy));
    CHECK(pp_device_free(ctx, d_out));
    CHECK(pp_device_free(ctx, d_mid));
    CHECK(pp_device_free(ctx, d_in));
    CHECK(pp_host_free(h_out));
    CHECK(pp_host_free(h_in));
    CHECK(pp_ctx_destroy(ctx));
    return 0;
}
