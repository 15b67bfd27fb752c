"""ctypes binding of libpixpath.so (include/pixpath.h).

The library is the product: there is no CPU fallback.  If it is missing or
cannot be loaded, every entry point raises immediately (``NativeMissing``).
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PIXPATH_LIB", os.path.join(_HERE, "libpixpath.so"))

PP_OK = 0
ERRORS = {-1: "PP_ERR_INVALID", -2: "PP_ERR_HIP", -3: "PP_ERR_NOMEM", -4: "PP_ERR_UNSUPPORTED"}

# every symbol declared in include/pixpath.h
EXPORTS = (
    "pp_abi_version", "pp_last_error", "pp_ctx_create", "pp_ctx_destroy", "pp_plane_bytes",
    "pp_v210_linesize", "pp_scale_plan_create", "pp_scale_chain_plan_create", "pp_scale_plan_destroy", "pp_scale_plan_filter",
    "pp_scale_plan_path", "pp_scale_plan_stats", "pp_scale_execute", "pp_pad_execute", "pp_v210_pack", "pp_cpvs_execute", "pp_spinner_upload", "pp_stall_compose",
    "pp_siti", "pp_siti_ex", "pp_fps_map",
    "pp_device_alloc", "pp_device_free", "pp_host_alloc", "pp_host_free", "pp_stream_create",
    "pp_stream_destroy", "pp_stream_synchronize", "pp_event_create", "pp_event_destroy", "pp_event_record",
    "pp_stream_wait_event", "pp_event_synchronize", "pp_event_elapsed_ms", "pp_copy_async", "pp_copy2d_async",
    "pp_frames_copy_async", "pp_annexb_frame_sizes", "pp_ivf_frame_sizes",
    "pp_ffv1_encoder_create", "pp_ffv1_encoder_destroy", "pp_ffv1_extradata", "pp_ffv1_encode",
    "pp_ffv1_encode_packets", "pp_ffv1_encode_stats", "pp_ffv1_encoder_memory", "pp_ffv1_encoder_reserve",
    "pp_ffv1_decoder_create", "pp_ffv1_decoder_destroy", "pp_ffv1_decoder_format", "pp_ffv1_decoder_slices", "pp_ffv1_decode",
    "pp_ffv1_decoder_geometry", "pp_ffv1_decoder_info", "pp_ffv1_decoder_reset", "pp_ffv1_decode_group",
)
PP_COPY_H2D, PP_COPY_D2H, PP_COPY_D2D = 1, 2, 3
PP_NAL_H264, PP_NAL_H265 = 1, 2
PP_SITI_NORMALIZE = 1


class NativeMissing(RuntimeError):
    pass


class PixpathError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (%d): %s" % (ERRORS.get(code, "?"), code, msg))
        self.code = code


class pp_frames(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p * 3), ("linesize", ctypes.c_int64 * 3),
                ("frame_stride", ctypes.c_int64 * 3)]


_lib = None


def lib():
    """Load libpixpath.so once; raise NativeMissing if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeMissing("libpixpath.so not found at %s -- run `make -C processing-chain_amd` "
                            "(or __graft_entry__.build())" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, dbl = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_double
    fr = ctypes.POINTER(pp_frames)
    sig = {
        "pp_abi_version": (i32, []),
        "pp_last_error": (ctypes.c_char_p, []),
        "pp_ctx_create": (i32, [i32, ctypes.POINTER(vp)]),
        "pp_ctx_destroy": (i32, [vp]),
        "pp_plane_bytes": (i64, [i32, i32, i32, i32, i64]),
        "pp_v210_linesize": (i64, [i32]),
        "pp_scale_plan_create": (i32, [vp, i32, i32, i32, i32, i32, i32, i32, dbl, dbl, ctypes.POINTER(vp)]),
        "pp_scale_chain_plan_create": (i32, [vp, i32, i32, i32, i32, i32, i32, i32, dbl, dbl, ctypes.POINTER(vp)]),
        "pp_scale_plan_destroy": (i32, [vp]),
        "pp_scale_plan_filter": (i32, [vp, i32, vp, vp, i32]),
        "pp_scale_plan_path": (i32, [vp]),
        "pp_scale_plan_stats": (i32, [vp, vp, i32]),
        "pp_scale_execute": (i32, [vp, fr, fr, i32, vp]),
        "pp_pad_execute": (i32, [vp, i32, i32, i32, fr, i32, i32, i32, i32, fr, i32, vp]),
        "pp_v210_pack": (i32, [vp, i32, i32, fr, fr, i32, vp]),
        "pp_cpvs_execute": (i32, [vp, i32, i32, i32, fr, i32, i32, i32, i32, i32, fr, i32, vp]),
        "pp_spinner_upload": (i32, [vp, i32, vp, i32, i32, i32]),
        "pp_stall_compose": (i32, [vp, i32, i32, i32, fr, vp, vp, fr, i32, vp]),
        "pp_siti": (i32, [vp, i32, i32, i32, vp, i64, i64, i32, vp, vp, vp, vp]),
        "pp_siti_ex": (i32, [vp, i32, i32, i32, vp, i64, i64, i32, vp, vp, vp, i32, vp]),
        "pp_fps_map": (i32, [i32, i64, i64, i64, i64, vp, i32]),
        "pp_device_alloc": (i32, [vp, i64, ctypes.POINTER(vp)]),
        "pp_device_free": (i32, [vp, vp]),
        "pp_host_alloc": (i32, [i64, ctypes.POINTER(vp)]),
        "pp_host_free": (i32, [vp]),
        "pp_stream_create": (i32, [vp, ctypes.POINTER(vp)]),
        "pp_stream_destroy": (i32, [vp, vp]),
        "pp_stream_synchronize": (i32, [vp]),
        "pp_event_create": (i32, [vp, ctypes.POINTER(vp)]),
        "pp_event_destroy": (i32, [vp]),
        "pp_event_record": (i32, [vp, vp]),
        "pp_stream_wait_event": (i32, [vp, vp]),
        "pp_event_synchronize": (i32, [vp]),
        "pp_event_elapsed_ms": (i32, [vp, vp, ctypes.POINTER(ctypes.c_float)]),
        "pp_copy_async": (i32, [vp, vp, i64, i32, vp]),
        "pp_copy2d_async": (i32, [vp, i64, vp, i64, i64, i64, i32, vp]),
        "pp_frames_copy_async": (i32, [i32, i32, i32, fr, fr, i32, i32, vp]),
        "pp_annexb_frame_sizes": (i64, [vp, i64, i32, vp, i64]),
        "pp_ivf_frame_sizes": (i64, [vp, i64, vp, i64, ctypes.POINTER(i64)]),
        "pp_ffv1_encoder_create": (i32, [vp, i32, i32, i32, i32, i32, i32, ctypes.POINTER(vp)]),
        "pp_ffv1_encoder_destroy": (i32, [vp]),
        "pp_ffv1_extradata": (i32, [vp, vp, i32]),
        "pp_ffv1_encode": (i64, [vp, fr, i32, vp, i64, vp, vp]),
        "pp_ffv1_encode_packets": (i64, [vp, fr, i32, vp, ctypes.POINTER(vp), vp]),
        "pp_ffv1_encode_stats": (i32, [vp, ctypes.POINTER(i32)]),
        "pp_ffv1_encoder_memory": (i32, [vp, ctypes.POINTER(i64)]),
        "pp_ffv1_encoder_reserve": (i32, [vp, i64]),
        "pp_ffv1_decoder_create": (i32, [vp, vp, i32, i32, i32, i32, ctypes.POINTER(vp)]),
        "pp_ffv1_decoder_destroy": (i32, [vp]),
        "pp_ffv1_decoder_format": (i32, [vp]),
        "pp_ffv1_decoder_slices": (i32, [vp, ctypes.POINTER(i32), ctypes.POINTER(i32)]),
        "pp_ffv1_decode": (i32, [vp, vp, vp, i32, fr, vp]),
        "pp_ffv1_decoder_geometry": (i32, [vp, ctypes.POINTER(i32), ctypes.POINTER(i32)]),
        "pp_ffv1_decoder_info": (i32, [vp, vp, i32]),
        "pp_ffv1_decoder_reset": (i32, [vp]),
        "pp_ffv1_decode_group": (i32, [vp, i32, vp, vp, vp, fr, vp]),
    }
    for name, (res, args) in sig.items():
        if "PIXPATH_LIB" in os.environ and not hasattr(L, name):
            continue  # an older measurement library (A/B runs): entry points it predates stay unbound
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(rc):
    if rc < 0:
        raise PixpathError(rc, lib().pp_last_error().decode(errors="replace"))
    return rc
