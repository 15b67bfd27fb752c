// Device / pinned-host memory, streams, events and copies of libpixpath.so
// (include/pixpath.h, "host transfer"): what a host without torch needs to
// drive decode -> H2D -> kernels -> D2H -> encode itself (SURVEY.md 8b:
// "pinned host alloc + async H2D/D2H on caller-supplied streams").  Thin
// wrappers over the HIP runtime with the library's error convention.
#include "common.hpp"

namespace {

hipMemcpyKind copy_kind(int kind) {
    switch (kind) {
    case PP_COPY_H2D: return hipMemcpyHostToDevice;
    case PP_COPY_D2H: return hipMemcpyDeviceToHost;
    case PP_COPY_D2D: return hipMemcpyDeviceToDevice;
    default: return hipMemcpyDefault;
    }
}

}  // namespace

extern "C" int pp_device_alloc(pp_ctx *ctx, int64_t bytes, void **out) {
    if (!ctx || !out || bytes < 0) PP_FAIL(PP_ERR_INVALID, "bad argument");
    *out = nullptr;
    if (bytes == 0) return PP_OK;
    PP_HIP(hipSetDevice(ctx->device));
    if (hipMalloc(out, (size_t)bytes) != hipSuccess) {
        *out = nullptr;
        PP_FAIL(PP_ERR_NOMEM, "device allocation of %lld bytes failed", (long long)bytes);
    }
    return PP_OK;
}

extern "C" int pp_device_free(pp_ctx *ctx, void *ptr) {
    if (!ctx) PP_FAIL(PP_ERR_INVALID, "null context");
    if (!ptr) return PP_OK;
    PP_HIP(hipSetDevice(ctx->device));
    PP_HIP(hipFree(ptr));
    return PP_OK;
}

extern "C" int pp_host_alloc(int64_t bytes, void **out) {
    if (!out || bytes < 0) PP_FAIL(PP_ERR_INVALID, "bad argument");
    *out = nullptr;
    if (bytes == 0) return PP_OK;
    if (hipHostMalloc(out, (size_t)bytes, hipHostMallocDefault) != hipSuccess) {
        *out = nullptr;
        PP_FAIL(PP_ERR_NOMEM, "pinned host allocation of %lld bytes failed", (long long)bytes);
    }
    return PP_OK;
}

extern "C" int pp_host_free(void *ptr) {
    if (!ptr) return PP_OK;
    PP_HIP(hipHostFree(ptr));
    return PP_OK;
}

extern "C" int pp_stream_create(pp_ctx *ctx, void **out) {
    if (!ctx || !out) PP_FAIL(PP_ERR_INVALID, "bad argument");
    PP_HIP(hipSetDevice(ctx->device));
    hipStream_t s = nullptr;
    PP_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *out = s;
    return PP_OK;
}

extern "C" int pp_stream_destroy(pp_ctx *ctx, void *stream) {
    if (!ctx) PP_FAIL(PP_ERR_INVALID, "null context");
    if (!stream) return PP_OK;
    PP_HIP(hipSetDevice(ctx->device));
    PP_HIP(hipStreamDestroy(static_cast<hipStream_t>(stream)));
    return PP_OK;
}

extern "C" int pp_stream_synchronize(void *stream) {
    PP_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    return PP_OK;
}

extern "C" int pp_event_create(pp_ctx *ctx, void **out) {
    if (!ctx || !out) PP_FAIL(PP_ERR_INVALID, "bad argument");
    PP_HIP(hipSetDevice(ctx->device));
    hipEvent_t e = nullptr;
    PP_HIP(hipEventCreate(&e));
    *out = e;
    return PP_OK;
}

extern "C" int pp_event_destroy(void *event) {
    if (!event) return PP_OK;
    PP_HIP(hipEventDestroy(static_cast<hipEvent_t>(event)));
    return PP_OK;
}

extern "C" int pp_event_record(void *event, void *stream) {
    if (!event) PP_FAIL(PP_ERR_INVALID, "null event");
    PP_HIP(hipEventRecord(static_cast<hipEvent_t>(event), static_cast<hipStream_t>(stream)));
    return PP_OK;
}

extern "C" int pp_stream_wait_event(void *stream, void *event) {
    if (!event) PP_FAIL(PP_ERR_INVALID, "null event");
    PP_HIP(hipStreamWaitEvent(static_cast<hipStream_t>(stream), static_cast<hipEvent_t>(event), 0));
    return PP_OK;
}

extern "C" int pp_event_synchronize(void *event) {
    if (!event) PP_FAIL(PP_ERR_INVALID, "null event");
    PP_HIP(hipEventSynchronize(static_cast<hipEvent_t>(event)));
    return PP_OK;
}

extern "C" int pp_event_elapsed_ms(void *start, void *end, float *ms) {
    if (!start || !end || !ms) PP_FAIL(PP_ERR_INVALID, "bad argument");
    PP_HIP(hipEventElapsedTime(ms, static_cast<hipEvent_t>(start), static_cast<hipEvent_t>(end)));
    return PP_OK;
}

extern "C" int pp_copy_async(void *dst, const void *src, int64_t bytes, int kind, void *stream) {
    if ((!dst || !src) && bytes) PP_FAIL(PP_ERR_INVALID, "null pointer");
    if (bytes < 0 || kind < PP_COPY_H2D || kind > PP_COPY_D2D) PP_FAIL(PP_ERR_INVALID, "bad size / kind");
    if (!bytes) return PP_OK;
    PP_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, copy_kind(kind), static_cast<hipStream_t>(stream)));
    return PP_OK;
}

extern "C" int pp_copy2d_async(void *dst, int64_t dpitch, const void *src, int64_t spitch, int64_t width_bytes,
                               int64_t rows, int kind, void *stream) {
    if ((!dst || !src) && rows && width_bytes) PP_FAIL(PP_ERR_INVALID, "null pointer");
    if (width_bytes < 0 || rows < 0 || dpitch < width_bytes || spitch < width_bytes || kind < PP_COPY_H2D ||
        kind > PP_COPY_D2D)
        PP_FAIL(PP_ERR_INVALID, "bad pitch / size / kind");
    if (!rows || !width_bytes) return PP_OK;
    PP_HIP(hipMemcpy2DAsync(dst, (size_t)dpitch, src, (size_t)spitch, (size_t)width_bytes, (size_t)rows,
                            copy_kind(kind), static_cast<hipStream_t>(stream)));
    return PP_OK;
}

// Every plane of every frame between two layouts of one format (e.g. a dense
// frame-interleaved pinned host batch and a pitched device batch): one 2-D
// copy per plane when both sides stack their frames' rows evenly, else one
// per plane and frame.
extern "C" int pp_frames_copy_async(int fmt, int w, int h, const pp_frames *dst, const pp_frames *src, int nframes,
                                    int kind, void *stream) {
    if (!dst || !src || nframes < 0 || w < 1 || h < 1) PP_FAIL(PP_ERR_INVALID, "bad argument");
    const pp::FmtInfo fi = pp::fmt_info(fmt);
    if (!fi.valid) PP_FAIL(PP_ERR_INVALID, "unknown format %d", fmt);
    const int planes = fi.packed ? 1 : 3;
    for (int p = 0; p < planes; ++p) {
        int64_t row_bytes, rows;
        if (fi.packed) {
            row_bytes = fmt == PP_FMT_V210 ? pp_v210_linesize(w) : 2LL * w;
            rows = h;
        } else {
            const int pw = p ? pp::ceil_rshift(w, fi.hsub) : w;
            row_bytes = (int64_t)pw * (fi.depth > 8 ? 2 : 1);
            rows = p ? pp::ceil_rshift(h, fi.vsub) : h;
        }
        const bool even = nframes < 2 || (dst->frame_stride[p] == dst->linesize[p] * rows &&
                                          src->frame_stride[p] == src->linesize[p] * rows);
        if (even) {
            int rc = pp_copy2d_async(dst->data[p], dst->linesize[p], src->data[p], src->linesize[p], row_bytes,
                                     rows * nframes, kind, stream);
            if (rc) return rc;
        } else {
            for (int f = 0; f < nframes; ++f) {
                int rc = pp_copy2d_async(static_cast<uint8_t *>(dst->data[p]) + f * dst->frame_stride[p],
                                         dst->linesize[p],
                                         static_cast<const uint8_t *>(src->data[p]) + f * src->frame_stride[p],
                                         src->linesize[p], row_bytes, rows, kind, stream);
                if (rc) return rc;
            }
        }
    }
    return PP_OK;
}
