// Context, error reporting and host helpers of libpixpath.so (include/pixpath.h).
#include <cstring>

#include "common.hpp"

namespace pp {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

}  // namespace pp

extern "C" int pp_abi_version(void) { return PP_ABI_VERSION; }

extern "C" const char *pp_last_error(void) { return pp::g_err; }

extern "C" int pp_ctx_create(int device, pp_ctx **out) {
    if (!out) PP_FAIL(PP_ERR_INVALID, "null argument");
    *out = nullptr;
    int n = 0;
    PP_HIP(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) PP_FAIL(PP_ERR_INVALID, "device %d of %d", device, n);
    PP_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    PP_HIP(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        PP_FAIL(PP_ERR_UNSUPPORTED, "libpixpath is built for gfx950, device %d is %s", device, prop.gcnArchName);
    pp_ctx *c = new pp_ctx();
    c->device = device;
    c->cus = prop.multiProcessorCount;
    *out = c;
    return PP_OK;
}

extern "C" int pp_ctx_destroy(pp_ctx *ctx) {
    if (!ctx) return PP_OK;
    if (ctx->spin_buf) {
        (void)hipSetDevice(ctx->device);
        (void)hipFree(ctx->spin_buf);
    }
    delete ctx;
    return PP_OK;
}

extern "C" int64_t pp_plane_bytes(int fmt, int w, int h, int plane, int64_t linesize) {
    const pp::FmtInfo fi = pp::fmt_info(fmt);
    if (!fi.valid || plane < 0 || plane > 2 || w < 1 || h < 1) return -1;
    if (fi.packed) return plane == 0 ? linesize * h : 0;
    const int ph = plane ? pp::ceil_rshift(h, fi.vsub) : h;
    return linesize * ph;
}

// vf_fps (libavfilter/vf_fps.c, rounding=near, eof_action=round): output frame
// k shows the last input frame whose timestamp rounds to <= k; the stream ends
// at round(n_in * out_rate / in_rate).
extern "C" int pp_fps_map(int n_in, int64_t in_num, int64_t in_den, int64_t out_num, int64_t out_den, int32_t *map,
                          int capacity) {
    if (n_in < 0 || in_num <= 0 || in_den <= 0 || out_num <= 0 || out_den <= 0 || (!map && capacity))
        PP_FAIL(PP_ERR_INVALID, "bad rate / arguments");
    const __int128 N = (__int128)in_den * out_num, D = (__int128)in_num * out_den;
    const __int128 n_out = ((__int128)n_in * N + D / 2) / D;
    if (n_out > capacity) PP_FAIL(PP_ERR_INVALID, "capacity %d < %lld output frames", capacity, (long long)n_out);
    int i = 0;
    for (int64_t k = 0; k < (int64_t)n_out; ++k) {
        while (i + 1 < n_in && ((__int128)(i + 1) * N * 2 + D) / (2 * D) <= k) ++i;
        map[k] = i;
    }
    return (int)n_out;
}
