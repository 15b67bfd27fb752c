"""ctypes front of oracle/ffv1_oracle.c (TEST INFRASTRUCTURE ONLY: tests/,
bench.py's cpu_baseline).  FFV1 v3 restatement, parity unpinned against
FFmpeg (absent); see the C file's header."""
import ctypes
import os

import numpy as np

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libpixoracle.so")
_lib = None
INFO_KEYS = ("version", "micro_version", "coder_type", "colorspace", "bits", "chroma_planes", "hsub", "vsub",
             "extra_plane", "num_h_slices", "num_v_slices", "quant_table_sets", "ec", "intra", "context_count",
             "crc_ok")


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(_LIB)
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
        L.ffv1o_extradata.argtypes = [i32, i32, i32, i32, i32, vp, i64]
        L.ffv1o_extradata.restype = i64
        L.ffv1o_encode_frame.argtypes = [vp, vp, i32, i32, i32, i32, i32, i32, i32, vp, i64]
        L.ffv1o_encode_frame.restype = i64
        L.ffv1o_decode_frame.argtypes = [vp, i64, vp, i64, i32, i32, vp, vp]
        L.ffv1o_decode_frame.restype = i32
        L.ffv1o_parse_extradata.argtypes = [vp, i64, vp]
        L.ffv1o_crc.argtypes = [ctypes.c_uint32, vp, i64]
        L.ffv1o_crc.restype = ctypes.c_uint32
        L.ffv1o_state_tables.argtypes = [vp, vp]
        _lib = L
    return _lib


def _ptrs(planes):
    arr = (ctypes.c_void_p * 3)(*[p.ctypes.data for p in planes])
    ls = (ctypes.c_int64 * 3)(*[p.strides[0] for p in planes])
    return arr, ls


def extradata(bits, hsub, vsub, nh, nv):
    buf = np.zeros(4096, np.uint8)
    n = lib().ffv1o_extradata(bits, hsub, vsub, nh, nv, buf.ctypes.data, buf.size)
    if n < 0:
        raise RuntimeError("extradata")
    return buf[:n].tobytes()


def parse_extradata(x):
    info = (ctypes.c_int * 16)()
    b = np.frombuffer(x, np.uint8)
    rc = lib().ffv1o_parse_extradata(b.ctypes.data, b.size, info)
    return rc, dict(zip(INFO_KEYS, list(info)))


def encode_frame(planes, bits, hsub, vsub, nh, nv):
    """planes: 2-D numpy arrays (uint8 / uint16).  Returns the packet bytes."""
    planes = [np.ascontiguousarray(p) for p in planes]
    h, w = planes[0].shape
    cap = sum(p.nbytes for p in planes) * 2 + 4096 + 64 * nh * nv
    out = np.zeros(cap, np.uint8)
    arr, ls = _ptrs(planes)
    n = lib().ffv1o_encode_frame(arr, ls, w, h, bits, hsub, vsub, nh, nv, out.ctypes.data, cap)
    if n < 0:
        raise RuntimeError("encode overflow")
    return out[:n].tobytes()


def decode_frame(extra, pkt, w, h, bits, hsub, vsub):
    """Returns (rc, planes)."""
    dt = np.uint16 if bits > 8 else np.uint8
    cw, ch = -(-w >> hsub), -(-h >> vsub)
    planes = [np.zeros((h, w), dt), np.zeros((ch, cw), dt), np.zeros((ch, cw), dt)]
    arr, ls = _ptrs(planes)
    x = np.frombuffer(extra, np.uint8)
    p = np.frombuffer(pkt, np.uint8)
    rc = lib().ffv1o_decode_frame(x.ctypes.data, x.size, p.ctypes.data, p.size, w, h, arr, ls)
    return rc, planes


def crc(data):
    b = np.frombuffer(bytes(data), np.uint8)
    return lib().ffv1o_crc(0, b.ctypes.data, b.size)
