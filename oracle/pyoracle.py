"""ctypes front-end of oracle/lib/libpixoracle.so (the C restatement).

TEST INFRASTRUCTURE ONLY -- see the header of oracle/pixoracle.c.  Planes are
numpy arrays (uint8 for 8-bit, uint16 for 10-bit formats), one 2-D array per
plane; packed outputs (uyvy422, v210) are 2-D uint8 arrays [rows, bytes].
"""
import ctypes
import os
import subprocess
from fractions import Fraction

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# PIXORACLE_LIB: another build of the same sources (bench.py's cpu_baseline
# times a -march=native build beside this scalar one)
_LIB_PATH = os.environ.get("PIXORACLE_LIB") or os.path.join(_HERE, "lib", "libpixoracle.so")

# format ids (same numbering as include/pixpath.h PP_FMT_*)
YUV420P, YUV422P, YUV444P, YUV420P10LE, YUV422P10LE, YUV444P10LE, UYVY422, V210 = range(8)
FMT_BY_NAME = {
    "yuv420p": YUV420P, "yuv422p": YUV422P, "yuv444p": YUV444P,
    "yuv420p10le": YUV420P10LE, "yuv422p10le": YUV422P10LE, "yuv444p10le": YUV444P10LE,
    "uyvy422": UYVY422, "v210": V210,
}
SWS_BILINEAR, SWS_BICUBIC, SWS_LANCZOS = 2, 4, 0x200
PARAM_DEFAULT = 123456.0


def fmt_info(fmt):
    """(depth, hsub, vsub) of a planar format id."""
    depth = 10 if fmt in (YUV420P10LE, YUV422P10LE, YUV444P10LE) else 8
    hsub = 0 if fmt in (YUV444P, YUV444P10LE) else 1
    vsub = 1 if fmt in (YUV420P, YUV420P10LE) else 0
    return depth, hsub, vsub


def plane_shapes(fmt, w, h):
    depth, hs, vs = fmt_info(fmt)
    cw, ch = -((-w) >> hs), -((-h) >> vs)
    return [(h, w), (ch, cw), (ch, cw)]


def plane_dtype(fmt):
    return np.uint16 if fmt_info(fmt)[0] > 8 else np.uint8


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i64p = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)
        L.po_sws_init.restype = vp
        L.po_sws_init.argtypes = [ctypes.c_int] * 7 + [ctypes.c_double] * 2
        L.po_sws_free.argtypes = [vp]
        L.po_sws_get_filter.argtypes = [vp, ctypes.c_int, vp, vp]
        L.po_sws_filter_size.argtypes = [vp, ctypes.c_int]
        L.po_sws_scale.argtypes = [vp, vp, vp, vp, vp]
        L.po_sws_scale_n.argtypes = [vp, vp, vp, vp, vp, ctypes.c_int]
        L.po_init_filter.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_int)] + [ctypes.c_int] * 6 + \
            [ctypes.c_double] * 2 + [ctypes.c_int] * 2
        L.po_pad.argtypes = [ctypes.c_int, vp, vp, ctypes.c_int, ctypes.c_int, vp, vp] + [ctypes.c_int] * 4
        L.po_v210_linesize.restype = ctypes.c_int64
        L.po_v210_linesize.argtypes = [ctypes.c_int]
        L.po_v210_pack.argtypes = [vp, ctypes.c_int64, vp, ctypes.c_int64, vp, ctypes.c_int64,
                                   ctypes.c_int, ctypes.c_int, vp, ctypes.c_int64]
        L.po_fps_map.argtypes = [ctypes.c_int] + [ctypes.c_int64] * 4 + [vp, ctypes.c_int]
        L.po_si_frame.restype = ctypes.c_double
        L.po_si_frame.argtypes = [vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.po_ti_frame.restype = ctypes.c_double
        L.po_ti_frame.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.po_siti_batch.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int, vp, vp, vp]
        L.po_spinner_to_yuva.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, vp, vp, vp, vp, vp]
        L.po_overlay_spinner.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, vp, vp, vp, vp, vp, ctypes.c_int, ctypes.c_int]
        _lib = L
    return _lib


def _ptrs(arrs):
    return (ctypes.c_void_p * 3)(*[a.ctypes.data for a in arrs])


def _lses(arrs):
    return (ctypes.c_int64 * 3)(*[a.strides[0] for a in arrs])


def init_filter(xinc, src_w, dst_w, align, one, flags, p0=PARAM_DEFAULT, p1=PARAM_DEFAULT,
                src_pos=128, dst_pos=128):
    """Raw initFilter(): returns (coef[dst_w, size] int16, pos[dst_w] int32)."""
    coef = np.zeros(dst_w * 64, dtype=np.int16)
    pos = np.zeros(dst_w, dtype=np.int32)
    size = ctypes.c_int(0)
    rc = lib().po_init_filter(coef.ctypes.data, pos.ctypes.data, ctypes.byref(size), xinc, src_w,
                              dst_w, align, one, flags, p0, p1, src_pos, dst_pos)
    if rc:
        raise ValueError("initFilter failed")
    return coef[: dst_w * size.value].reshape(dst_w, size.value).copy(), pos


class Sws:
    """One swscale context (sws_init_context restatement)."""

    def __init__(self, src_fmt, sw, sh, dst_fmt, dw, dh, flags=SWS_BICUBIC,
                 p0=PARAM_DEFAULT, p1=PARAM_DEFAULT):
        self.src_fmt, self.dst_fmt = src_fmt, dst_fmt
        self.sw, self.sh, self.dw, self.dh = sw, sh, dw, dh
        self._h = lib().po_sws_init(src_fmt, sw, sh, dst_fmt, dw, dh, flags, p0, p1)
        if not self._h:
            raise ValueError("unsupported conversion")

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            try:
                _lib.po_sws_free(self._h)
            except Exception:
                pass
            self._h = None

    def filter(self, which):
        """which: 0 luma-H, 1 chroma-H, 2 luma-V, 3 chroma-V -> (coef, pos) or None."""
        size = lib().po_sws_filter_size(self._h, which)
        if size <= 0:
            return None
        if which in (0, 2):
            n = self.dw if which == 0 else self.dh
        else:
            shapes = plane_shapes(self.dst_fmt if self.dst_fmt != UYVY422 else YUV422P, self.dw, self.dh)
            n = shapes[1][1] if which == 1 else shapes[1][0]
        coef = np.zeros((n, size), dtype=np.int16)
        pos = np.zeros(n, dtype=np.int32)
        lib().po_sws_get_filter(self._h, which, coef.ctypes.data, pos.ctypes.data)
        return coef, pos

    def scale(self, planes):
        planes = [np.ascontiguousarray(p) for p in planes]
        if self.dst_fmt == UYVY422:
            out = [np.zeros((self.dh, 2 * self.dw), dtype=np.uint8)] * 1
            outs = out + [out[0], out[0]]
        else:
            outs = [np.zeros(s, dtype=plane_dtype(self.dst_fmt))
                    for s in plane_shapes(self.dst_fmt, self.dw, self.dh)]
        rc = lib().po_sws_scale(self._h, _ptrs(planes), _lses(planes), _ptrs(outs), _lses(outs))
        if rc:
            raise RuntimeError("po_sws_scale failed")
        return outs[:1] if self.dst_fmt == UYVY422 else outs

    def out_planes(self):
        """Output planes for scale_into (planar destination formats)."""
        return [np.zeros(s, dtype=plane_dtype(self.dst_fmt)) for s in plane_shapes(self.dst_fmt, self.dw, self.dh)]

    def scale_into(self, planes, outs, count=1):
        """Scale the same frame `count` times into preallocated planar `outs`
        (bench.py's cpu_baseline: one C call per batch, no per-frame Python)."""
        if lib().po_sws_scale_n(self._h, _ptrs(planes), _lses(planes), _ptrs(outs), _lses(outs), int(count)):
            raise RuntimeError("po_sws_scale failed")


def scale(src_fmt, planes, dst_fmt, dw, dh, flags=SWS_BICUBIC, p0=PARAM_DEFAULT, p1=PARAM_DEFAULT):
    sh, sw = planes[0].shape
    return Sws(src_fmt, sw, sh, dst_fmt, dw, dh, flags, p0, p1).scale(planes)


def pad(fmt, planes, dw, dh, x, y):
    planes = [np.ascontiguousarray(p) for p in planes]
    sh, sw = planes[0].shape
    outs = [np.zeros(s, dtype=plane_dtype(fmt)) for s in plane_shapes(fmt, dw, dh)]
    if lib().po_pad(fmt, _ptrs(planes), _lses(planes), sw, sh, _ptrs(outs), _lses(outs), dw, dh, x, y):
        raise ValueError("pad out of range")
    return outs


def v210_linesize(w):
    return lib().po_v210_linesize(w)


def v210_pack(planes):
    Y, U, V = [np.ascontiguousarray(p, dtype=np.uint16) for p in planes]
    h, w = Y.shape
    ls = v210_linesize(w)
    out = np.zeros((h, ls), dtype=np.uint8)
    lib().po_v210_pack(Y.ctypes.data, Y.strides[0], U.ctypes.data, U.strides[0], V.ctypes.data,
                       V.strides[0], w, h, out.ctypes.data, ls)
    return out


def fps_map(n_in, in_rate, out_rate):
    in_rate, out_rate = Fraction(in_rate), Fraction(out_rate)
    cap = int(n_in * out_rate / in_rate) + 4
    m = np.zeros(cap, dtype=np.int32)
    n = lib().po_fps_map(n_in, in_rate.numerator, in_rate.denominator, out_rate.numerator,
                         out_rate.denominator, m.ctypes.data, cap)
    return m[:n].copy()


def siti_c(frames, bitdepth, prev=None):
    frames = np.ascontiguousarray(frames)
    n, h, w = frames.shape
    si = np.zeros(n)
    ti = np.zeros(n)
    pp = None
    if prev is not None:
        prev = np.ascontiguousarray(prev, dtype=frames.dtype)
        pp = prev.ctypes.data
    lib().po_siti_batch(frames.ctypes.data, frames.strides[1], frames.strides[0], n, w, h, bitdepth,
                        pp, si.ctypes.data, ti.ctypes.data)
    return si, ti


def spinner_to_yuva(rgba, fmt):
    depth, hs, vs = fmt_info(fmt)
    rgba = np.ascontiguousarray(rgba, dtype=np.uint8)
    h, w = rgba.shape[:2]
    Y = np.zeros((h, w), np.uint16)
    Al = np.zeros((h, w), np.uint16)
    U = np.zeros((h >> vs, w >> hs), np.uint16)
    V = np.zeros_like(U)
    Ac = np.zeros_like(U)
    if lib().po_spinner_to_yuva(rgba.ctypes.data, w, h, hs, vs, depth, Y.ctypes.data, Al.ctypes.data,
                                U.ctypes.data, V.ctypes.data, Ac.ctypes.data):
        raise ValueError("spinner size not on the chroma grid")
    return Y, Al, U, V, Ac


def overlay_spinner(fmt, planes, yuva):
    depth, hs, vs = fmt_info(fmt)
    outs = [np.array(p, copy=True, order="C") for p in planes]
    H, W = outs[0].shape
    Y, Al, U, V, Ac = yuva
    lib().po_overlay_spinner(_ptrs(outs), _lses(outs), W, H, hs, vs, depth, Y.ctypes.data,
                             Al.ctypes.data, U.ctypes.data, V.ctypes.data, Ac.ctypes.data,
                             Y.shape[1], Y.shape[0])
    return outs
