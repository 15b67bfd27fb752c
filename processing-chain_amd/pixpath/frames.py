"""Device frame batches: HBM layout of N frames of one pixel format.

Each plane is one torch tensor [N, rows, pitch] (uint8 for 8-bit / packed
formats, uint16 for 10-bit), so a whole batch is a few large contiguous
allocations: plane p of frame f lives at data[p] + f * frame_stride[p].  The
pitch is rounded up to 16 bytes so every row start is 16-B aligned (the
kernels' vector path).  torch is used only as the device allocator.
"""
import numpy as np
import torch

from . import formats
from ._native import pp_frames


import os

from . import _native


def _layout_pad():
    """Layout padding for measurements (tools/gpu_pad_sweep.sh: bytes added to
    every row pitch, rows added to every plane of a frame; the kernels take any
    pitch / frame stride).  Read only when a library other than the product's
    is loaded (PIXPATH_LIB = the measurement build), like the library's own
    knobs: the product layout never depends on the environment."""
    if os.path.realpath(_native.LIB_PATH) == os.path.realpath(os.path.join(os.path.dirname(_native.__file__),
                                                                          "libpixpath.so")):
        return 0, 0
    return int(os.environ.get("PIXPATH_PITCH_PAD", "0")), int(os.environ.get("PIXPATH_ROWS_PAD", "0"))


_PITCH_PAD, _ROWS_PAD = _layout_pad()


def _pitch(cols, bps, align=16):
    b = cols * bps + _PITCH_PAD
    return ((b + align - 1) // align * align) // bps


class FrameBatch:
    def __init__(self, f, w, h, n, device="cuda", planes=None, zero=False):
        self.fmt = formats.fmt(f)
        self.w, self.h, self.n = int(w), int(h), int(n)
        self.shapes = formats.plane_shapes(self.fmt, w, h)
        bps = 1 if self.fmt.packed else self.fmt.bytes_per_sample
        dtype = torch.uint16 if bps == 2 else torch.uint8
        if planes is None:
            alloc = torch.zeros if zero else torch.empty
            planes = [alloc((self.n, r + _ROWS_PAD, _pitch(c, bps)), dtype=dtype, device=device)
                      for r, c in self.shapes]
        self.planes = planes
        self.bps = bps

    @classmethod
    def interleaved(cls, f, w, h, n, device="cuda", storage=None):
        """Frame-interleaved batch: one [n, frame_bytes] uint8 buffer holding dense
        Y|U|V frames (the raw pipe / pinned-buffer layout), planes as strided views.
        One contiguous H2D/D2H copy moves the whole batch."""
        fm = formats.fmt(f)
        fb = formats.frame_bytes(fm, w, h)
        if storage is None:
            storage = torch.empty((n, fb), dtype=torch.uint8, device=device)
        flat = storage.reshape(-1)
        shapes = formats.plane_shapes(fm, w, h)
        bps = 1 if fm.packed else fm.bytes_per_sample
        base = flat.view(torch.uint16) if bps == 2 else flat
        planes, off = [], 0
        so = base.storage_offset()  # as_strided's offset is absolute: keep a sliced storage's own
        for r, c in shapes:
            planes.append(base.as_strided((n, r, c), (fb // bps, c, 1), so + off // bps))
            off += r * c * bps
        b = cls(fm, w, h, n, device=device, planes=planes)
        b.storage = storage
        return b

    @property
    def device(self):
        return self.planes[0].device

    def view(self, p):
        """Plane p without the pitch padding: [N, rows, cols]."""
        r, c = self.shapes[p]
        return self.planes[p][:, :r, :c]

    def frames_struct(self, first=0):
        s = pp_frames()
        for p in range(3):
            t = self.planes[min(p, len(self.planes) - 1)]
            es = t.element_size()
            s.data[p] = t.data_ptr() + first * t.stride(0) * es
            s.linesize[p] = t.stride(1) * es
            s.frame_stride[p] = t.stride(0) * es
        return s

    # ---- host transfer helpers (tests / CLI) ----
    @classmethod
    def from_numpy(cls, f, planes_np, device="cuda"):
        """planes_np: list of [N, rows, cols] numpy arrays (or [rows, cols] for N=1)."""
        arrs = [np.asarray(a) for a in planes_np]
        if arrs[0].ndim == 2:
            arrs = [a[None] for a in arrs]
        n, h = arrs[0].shape[0], arrs[0].shape[1]
        fm = formats.fmt(f)
        w = arrs[0].shape[2] // 2 if fm.id == formats.UYVY422 else arrs[0].shape[2]
        if fm.id == formats.V210:
            raise ValueError("v210 input batches are not supported")
        b = cls(fm, w, h, n, device=device)
        for p, a in enumerate(arrs):
            r, c = b.shapes[p]
            if a.shape[1:] != (r, c):
                raise ValueError("plane %d shape %s != %s" % (p, a.shape[1:], (r, c)))
            t = torch.from_numpy(np.ascontiguousarray(a.astype(np.uint16 if b.bps == 2 else np.uint8)))
            b.planes[p][:, :r, :c].copy_(t.to(device))
        return b

    def to_numpy(self):
        """List of [N, rows, cols] numpy arrays."""
        return [self.view(p).cpu().numpy() for p in range(len(self.planes))]
