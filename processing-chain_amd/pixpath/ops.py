"""Python face of the HIP pixel path (thin wrappers over include/pixpath.h).

Every function enqueues on the current torch stream of the frames' device
(or an explicit ``stream``) and returns without synchronising.  There is no
CPU fallback: a missing libpixpath.so raises ``NativeMissing``.
"""
import ctypes
from fractions import Fraction

import numpy as np
import torch

from . import formats
from ._native import check, lib
from .frames import FrameBatch

FLAGS = {"bilinear": 0x2, "bicubic": 0x4, "lanczos": 0x200}
PARAM_DEFAULT = 123456.0
PLAN_GENERIC = 0x10000000  # PP_PLAN_GENERIC (ABI v5)

_contexts = {}


class Context:
    """One pp_ctx per process and device (the one-process-per-GPU model)."""

    def __init__(self, device=0):
        h = ctypes.c_void_p()
        check(lib().pp_ctx_create(int(device), ctypes.byref(h)))
        self.handle = h
        self.device = int(device)

    def __del__(self):
        if getattr(self, "handle", None) and lib is not None:
            try:
                lib().pp_ctx_destroy(self.handle)
            except Exception:
                pass
            self.handle = None


def context(device=None):
    if device is None:
        device = torch.cuda.current_device()
    if isinstance(device, torch.device):
        device = device.index if device.index is not None else torch.cuda.current_device()
    device = int(device)
    if device not in _contexts:
        _contexts[device] = Context(device)
    return _contexts[device]


def _stream(t, stream):
    if stream is not None:
        return ctypes.c_void_p(stream if isinstance(stream, int) else stream.cuda_stream)
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


class Scaler:
    """swscale-equivalent plan: `scale=W:H:flags=<f>` plus the -pix_fmt conversion.

    Mirrors the filter the reference requests at lib/ffmpeg.py:992 / :1038 /
    :1213 / :800.  flags: "bicubic" (the reference's), "lanczos", "bilinear".
    """

    def __init__(self, src_fmt, sw, sh, dst_fmt, dw, dh, flags="bicubic", param0=None, param1=None,
                 device=None, chain=False, generic=False):
        """chain=True: create_avpvs_segment's two stages (scale into the overlay's
        yuv420p, then yuv420p -> dst_fmt bicubic at the same size) as one plan
        (pp_scale_chain_plan_create): one launch when kernel_path > 0.
        generic=True: the general scale_kernel even where the strip kernel
        applies (PP_PLAN_GENERIC; both are bit-exact, tests run both)."""
        self.src_fmt, self.dst_fmt = formats.fmt(src_fmt), formats.fmt(dst_fmt)
        self.sw, self.sh, self.dw, self.dh = int(sw), int(sh), int(dw), int(dh)
        self.ctx = context(device)
        fl = FLAGS[flags] if isinstance(flags, str) else int(flags)
        if generic:
            fl |= PLAN_GENERIC
        h = ctypes.c_void_p()
        create = lib().pp_scale_chain_plan_create if chain else lib().pp_scale_plan_create
        check(create(
            self.ctx.handle, self.src_fmt.id, self.sw, self.sh, self.dst_fmt.id, self.dw, self.dh, fl,
            PARAM_DEFAULT if param0 is None else float(param0),
            PARAM_DEFAULT if param1 is None else float(param1), ctypes.byref(h)))
        self.handle = h

    def __del__(self):
        if getattr(self, "handle", None):
            try:
                lib().pp_scale_plan_destroy(self.handle)
            except Exception:
                pass
            self.handle = None

    @property
    def kernel_path(self):
        """> 0: the strip kernel runs (its H window in dwords); 0: the general kernel."""
        return check(lib().pp_scale_plan_path(self.handle))

    @property
    def stats(self):
        """Launch geometry (pp_scale_plan_stats) as a dict."""
        keys = ("lds_bytes", "threads", "tiles_per_frame", "cho", "seg_rows", "vtp_luma", "vtp_chroma",
                "staged_cols", "window_rows", "max_new_rows")
        v = np.zeros(len(keys), dtype=np.int64)
        n = check(lib().pp_scale_plan_stats(self.handle, v.ctypes.data, len(keys)))
        return dict(zip(keys[:n], (int(x) for x in v[:n])))

    def filter(self, which):
        """FFmpeg-layout filter (coef [n, size] int16, pos [n] int32) or None (unscaled path)."""
        n = [self.dw, -((-self.dw) >> (self.dst_fmt.hsub)), self.dh,
             -((-self.dh) >> (0 if self.dst_fmt.packed else self.dst_fmt.vsub))][which]
        cap = n * 64
        coef = np.zeros(cap, dtype=np.int16)
        pos = np.zeros(n, dtype=np.int32)
        size = check(lib().pp_scale_plan_filter(self.handle, which, coef.ctypes.data, pos.ctypes.data, cap))
        if size == 0:
            return None
        return coef[: n * size].reshape(n, size).copy(), pos

    def __call__(self, src, dst=None, stream=None):
        if (src.fmt.id, src.w, src.h) != (self.src_fmt.id, self.sw, self.sh):
            raise ValueError("source batch does not match the plan")
        if dst is None:
            dst = FrameBatch(self.dst_fmt, self.dw, self.dh, src.n, device=src.device)
        if (dst.fmt.id, dst.w, dst.h) != (self.dst_fmt.id, self.dw, self.dh) or dst.n < src.n:
            raise ValueError("destination batch does not match the plan")
        s, d = src.frames_struct(), dst.frames_struct()
        check(lib().pp_scale_execute(self.handle, ctypes.byref(s), ctypes.byref(d), src.n,
                                     _stream(src.planes[0], stream)))
        return dst


def pad(src, dw, dh, x=-1, y=-1, dst=None, stream=None):
    """vf_pad with the reference's centring (lib/ffmpeg.py:1183); x=y=-1 -> (ow-iw)/2."""
    ctx = context(src.device.index)
    if dst is None:
        dst = FrameBatch(src.fmt, dw, dh, src.n, device=src.device)
    s, d = src.frames_struct(), dst.frames_struct()
    check(lib().pp_pad_execute(ctx.handle, src.fmt.id, src.w, src.h, ctypes.byref(s), dw, dh, x, y,
                               ctypes.byref(d), src.n, _stream(src.planes[0], stream)))
    return dst


def v210_pack(src, dst=None, stream=None):
    """yuv422p10le -> v210 (libavcodec/v210enc.c), the PC CPVS codec for 10-bit AVPVS."""
    if src.fmt.id != formats.YUV422P10LE:
        raise ValueError("v210 packs yuv422p10le")
    ctx = context(src.device.index)
    if dst is None:
        dst = FrameBatch(formats.V210, src.w, src.h, src.n, device=src.device)
    s, d = src.frames_struct(), dst.frames_struct()
    check(lib().pp_v210_pack(ctx.handle, src.w, src.h, ctypes.byref(s), ctypes.byref(d), src.n,
                             _stream(src.planes[0], stream)))
    return dst


def cpvs(src, W=None, H=None, out_fmt=None, x=-1, y=-1, dst=None, stream=None):
    """Fused PC CPVS: pad to W x H (reference centring) + 4:2:0->4:2:2 + uyvy422
    (8-bit AVPVS) or v210 (10-bit) packing in one pass (lib/ffmpeg.py:1177-1201)."""
    W = src.w if W is None else int(W)
    H = src.h if H is None else int(H)
    if out_fmt is None:
        out_fmt = formats.UYVY422 if src.fmt.depth == 8 else formats.V210
    of = formats.fmt(out_fmt)
    ctx = context(src.device.index)
    if dst is None:
        dst = FrameBatch(of, W, H, src.n, device=src.device)
    s, d = src.frames_struct(), dst.frames_struct()
    check(lib().pp_cpvs_execute(ctx.handle, src.fmt.id, src.w, src.h, ctypes.byref(s), W, H, x, y, of.id,
                                ctypes.byref(d), src.n, _stream(src.planes[0], stream)))
    return dst


def siti(luma, bitdepth, prev=None, stream=None, normalize=False):
    """Per-frame P.910 SI/TI of a [N, H, W] luma tensor (uint8 / uint16, may be a
    pitched view).  Returns two float64 device tensors [N]; ti[0] is NaN when
    ``prev`` (the frame before luma[0]) is not given.  ``normalize``: values
    divided by 2^(bitdepth-8) (the 8-bit scale, PP_SITI_NORMALIZE)."""
    if luma.dim() != 3:
        raise ValueError("luma must be [N, H, W]")
    n, h, w = luma.shape
    es = luma.element_size()
    if luma.stride(2) != 1:
        raise ValueError("luma rows must be contiguous")
    ctx = context(luma.device.index)
    si = torch.empty(n, dtype=torch.float64, device=luma.device)
    ti = torch.empty(n, dtype=torch.float64, device=luma.device)
    pp = None
    if prev is not None:
        if prev.stride(-1) != 1 or prev.stride(-2) != luma.stride(1):
            raise ValueError("prev must share the luma row pitch")
        pp = ctypes.c_void_p(prev.data_ptr())
    check(lib().pp_siti_ex(ctx.handle, int(bitdepth), w, h, ctypes.c_void_p(luma.data_ptr()), luma.stride(1) * es,
                           luma.stride(0) * es, n, pp, ctypes.c_void_p(si.data_ptr()),
                           ctypes.c_void_p(ti.data_ptr()), 1 if normalize else 0, _stream(luma, stream)))
    return si, ti


def spinner_upload(rgba_frames, f, device=None):
    """Upload an RGBA8 animation [n, h, w, 4] (host) for stall compositing."""
    a = np.ascontiguousarray(rgba_frames, dtype=np.uint8)
    if a.ndim == 3:
        a = a[None]
    n, h, w, _ = a.shape
    ctx = context(device)
    check(lib().pp_spinner_upload(ctx.handle, formats.fmt(f).id, a.ctypes.data, n, w, h))


def stall_compose(src, src_index, spinner_index, dst=None, stream=None):
    """dst[k] = src[src_index[k]] (black if < 0) + spinner frame spinner_index[k] (none if < 0)."""
    si = np.ascontiguousarray(src_index, dtype=np.int32)
    sp = np.ascontiguousarray(spinner_index, dtype=np.int32)
    if si.shape != sp.shape:
        raise ValueError("index arrays differ in length")
    if si.size and (si.max() >= src.n):
        raise ValueError("source index out of range")
    ctx = context(src.device.index)
    if dst is None:
        dst = FrameBatch(src.fmt, src.w, src.h, si.size, device=src.device)
    s, d = src.frames_struct(), dst.frames_struct()
    check(lib().pp_stall_compose(ctx.handle, src.fmt.id, src.w, src.h, ctypes.byref(s), si.ctypes.data,
                                 sp.ctypes.data, ctypes.byref(d), si.size, _stream(src.planes[0], stream)))
    return dst


def fps_map(n_in, in_rate, out_rate):
    """vf_fps output->input frame indices (host, no GPU needed)."""
    a, b = Fraction(in_rate), Fraction(out_rate)
    cap = int(n_in * b / a) + 4
    m = np.zeros(max(cap, 1), dtype=np.int32)
    n = check(lib().pp_fps_map(int(n_in), a.numerator, a.denominator, b.numerator, b.denominator,
                               m.ctypes.data, cap))
    return m[:n].copy()
