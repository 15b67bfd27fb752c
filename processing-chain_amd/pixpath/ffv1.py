"""FFV1 encoder of the AVPVS intermediate on the MI355X (SURVEY.md section 8f
row 1): the pixel stage's output in the bitstream the reference's
`-c:v ffv1 -threads 4 -level 3 -coder 1 -context 1 -slicecrc 1`
(lib/ffmpeg.py:993, :1047) produces -- FFV1 version 3, range coder, slice
CRCs -- encoded by libpixpath's ffv1_slice_kernel (one lane per slice).

Bitstream choices that differ from ffmpeg's encoder and the parity status
(unpinned: no FFV1 decoder exists in this container or on the GPU box; the
CPU restatement oracle/ffv1_oracle.c decodes it losslessly) are in DESIGN.md.
"""
import ctypes

import numpy as np
import torch

from . import formats
from ._native import check, lib
from .ops import _stream, context


class Ffv1Encoder:
    def __init__(self, fmt, w, h, slices=(8, 8), max_frames=600, device=None, host_only=False):
        self.fmt = formats.fmt(fmt)
        self.w, self.h = int(w), int(h)
        self.slices = (int(slices[0]), int(slices[1]))
        self.max_frames = int(max_frames)
        self.ctx = None if host_only else context(device)
        h_ = ctypes.c_void_p()
        check(lib().pp_ffv1_encoder_create(None if host_only else self.ctx.handle, self.fmt.id, self.w, self.h,
                                           self.slices[0], self.slices[1], self.max_frames, ctypes.byref(h_)))
        self.handle = h_
        self._out = None

    def __del__(self):
        if getattr(self, "handle", None):
            try:
                lib().pp_ffv1_encoder_destroy(self.handle)
            except Exception:
                pass
            self.handle = None

    @property
    def extradata(self):
        """The configuration record (codec private data of the AVI/MKV stream)."""
        n = check(lib().pp_ffv1_extradata(self.handle, None, 0))
        buf = (ctypes.c_uint8 * n)()
        check(lib().pp_ffv1_extradata(self.handle, buf, n))
        return bytes(buf)

    def encode(self, src, stream=None):
        """Encode a FrameBatch; returns (device uint8 tensor of the packets back to back,
        numpy int64 frame sizes).  Synchronises the stream."""
        if (src.fmt.id, src.w, src.h) != (self.fmt.id, self.w, self.h):
            raise ValueError("batch does not match the encoder")
        raw = sum(src.view(p)[0].numel() * src.view(p).element_size() for p in range(3))
        cap = src.n * (raw * 3 // 2 + 4096 + 64 * self.slices[0] * self.slices[1])
        if self._out is None or self._out.numel() < cap:
            self._out = torch.empty(cap, dtype=torch.uint8, device=src.device)
        sizes = np.zeros(src.n, np.int64)
        s = src.frames_struct()
        total = check(lib().pp_ffv1_encode(self.handle, ctypes.byref(s), src.n,
                                           ctypes.c_void_p(self._out.data_ptr()), cap,
                                           sizes.ctypes.data_as(ctypes.c_void_p), _stream(src.planes[0], stream)))
        return self._out[:total], sizes

    def encode_to_host(self, src, stream=None):
        """List of per-frame packets (bytes)."""
        buf, sizes = self.encode(src, stream)
        data = buf.cpu().numpy().tobytes()
        out, off = [], 0
        for n in sizes.tolist():
            out.append(data[off:off + n])
            off += n
        return out


class Ffv1Decoder:
    """FFV1 v3 intra decoder on the GPU (one lane per slice): the AVPVS read
    back for the CPVS stage.  ``decode(packets, sizes)`` takes the frame
    packets back to back in host memory and returns a FrameBatch in HBM."""

    def __init__(self, extradata, w, h, max_frames=600, device=None, host_only=False):
        self.w, self.h, self.max_frames = int(w), int(h), int(max_frames)
        self.ctx = None if host_only else context(device)
        buf = (ctypes.c_uint8 * len(extradata)).from_buffer_copy(extradata)
        h_ = ctypes.c_void_p()
        check(lib().pp_ffv1_decoder_create(None if host_only else self.ctx.handle, buf, len(extradata), self.w,
                                           self.h, self.max_frames, ctypes.byref(h_)))
        self.handle = h_
        fid = check(lib().pp_ffv1_decoder_format(h_))
        self.fmt = formats.fmt(fid)

    def __del__(self):
        if getattr(self, "handle", None):
            try:
                lib().pp_ffv1_decoder_destroy(self.handle)
            except Exception:
                pass
            self.handle = None

    def decode(self, packets, sizes, dst=None, stream=None):
        from .frames import FrameBatch
        data = np.frombuffer(bytes(packets) if not isinstance(packets, (bytes, bytearray)) else packets, np.uint8)
        sizes = np.ascontiguousarray(sizes, dtype=np.int64)
        n = len(sizes)
        if dst is None:
            dst = FrameBatch(self.fmt, self.w, self.h, n, device=torch.device("cuda", self.ctx.device))
        s = dst.frames_struct()
        check(lib().pp_ffv1_decode(self.handle, data.ctypes.data_as(ctypes.c_void_p),
                                   sizes.ctypes.data_as(ctypes.c_void_p), n, ctypes.byref(s),
                                   _stream(dst.planes[0], stream)))
        return dst
