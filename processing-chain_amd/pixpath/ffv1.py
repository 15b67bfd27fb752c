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
        if isinstance(packets, np.ndarray):
            data = np.ascontiguousarray(packets, dtype=np.uint8)
        else:
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


class Ffv1AviWriter:
    """`cli avpvs --gpu-ffv1`: the AVPVS written as FFV1 encoded on the GPU in
    an AVI (pixpath.avi) -- the `-c:v ffv1 ... <pvs>.avi` of lib/ffmpeg.py:993
    without ffmpeg's encoder.  Takes dense host frames (the pipeline's writer
    interface), encodes them in batches."""

    def __init__(self, path, fmt, w, h, rate, slices=(8, 8), batch=64, device=None):
        from . import avi
        from .frames import FrameBatch
        self.fmt = formats.fmt(fmt)
        self.fb = formats.frame_bytes(self.fmt, w, h)
        self.batch = int(batch)
        self.enc = Ffv1Encoder(self.fmt, w, h, slices=slices, max_frames=self.batch, device=device)
        dev = torch.device("cuda", self.enc.ctx.device)
        self.stage = FrameBatch.interleaved(self.fmt, w, h, self.batch, device=dev)
        self.avi = avi.AviWriter(path, w, h, rate, extradata=self.enc.extradata)

    def write(self, frames_u8):
        from .frames import FrameBatch
        data = np.frombuffer(memoryview(frames_u8).cast("B"), np.uint8)
        n = len(data) // self.fb
        for i in range(0, n, self.batch):
            k = min(self.batch, n - i)
            self.stage.storage[:k].copy_(torch.from_numpy(data[i * self.fb:(i + k) * self.fb].reshape(k, self.fb)))
            src = FrameBatch.interleaved(self.fmt, self.enc.w, self.enc.h, k, device=self.stage.device,
                                         storage=self.stage.storage[:k])
            for p in self.enc.encode_to_host(src):
                self.avi.write_packet(p)

    def close(self):
        self.avi.close()


class Ffv1AviReader:
    """`cli cpvs --gpu-ffv1`: an FFV1 AVI (as Ffv1AviWriter writes it) read
    back through the GPU decoder; the reader interface of pixpath.io.  Only
    the packet index is held (pixpath.avi.scan); each batch's packets are read
    from the file when that batch is decoded, so a long-test AVPVS of tens of
    GB never sits in host memory."""

    def __init__(self, path, batch=256, device=None):
        from . import avi
        info, self.index = avi.scan(path)
        if info.get("fourcc") != b"FFV1":
            raise ValueError("%s: not an FFV1 AVI" % path)
        self.w, self.h, self.rate = info["w"], info["h"], info["rate"]
        self.batch = int(batch)
        self.dec = Ffv1Decoder(info["extradata"], self.w, self.h, max_frames=self.batch, device=device)
        self.fmt = self.dec.fmt
        self.pos = 0
        self.fh = open(path, "rb")

    @property
    def frame_bytes(self):
        return formats.frame_bytes(self.fmt, self.w, self.h)

    def __len__(self):
        return len(self.index)

    def _read(self, i, m):
        """Packets i..i+m-1 back to back (one read of their file span) and their sizes."""
        ent = self.index[i:i + m]
        lo, hi = ent[0][0], ent[-1][0] + ent[-1][1]
        self.fh.seek(lo)
        span = np.frombuffer(self.fh.read(hi - lo), np.uint8)
        sizes = np.array([s for _, s in ent], np.int64)
        if hi - lo == int(sizes.sum()):
            return span, sizes
        return np.concatenate([span[o - lo:o - lo + s] for o, s in ent]), sizes

    def read_device(self, n):
        """Decode up to n frames into an interleaved device FrameBatch (None at the end)."""
        from .frames import FrameBatch
        k = min(n, len(self.index) - self.pos)
        if k <= 0:
            return None
        out = FrameBatch.interleaved(self.fmt, self.w, self.h, k, device=torch.device("cuda", self.dec.ctx.device))
        done = 0
        while done < k:
            m = min(self.batch, k - done)
            data, sizes = self._read(self.pos, m)
            part = FrameBatch.interleaved(self.fmt, self.w, self.h, m, device=out.device,
                                          storage=out.storage[done:done + m])
            self.dec.decode(data, sizes, dst=part)
            self.pos += m
            done += m
        return out

    def read_into(self, buf, n):
        """Decode up to n frames into the dense host array buf [n, frame_bytes]; returns the count."""
        out = self.read_device(n)
        if out is None:
            return 0
        k = out.n
        buf[:k] = out.storage[:k].cpu().numpy()
        return k

    def close(self):
        self.fh.close()
