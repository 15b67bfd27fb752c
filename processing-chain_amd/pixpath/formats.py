"""Pixel formats of the reference's raw-frame path and their HBM layout.

AVPVS formats come from Segment.set_pix_fmt / Pvs.get_pix_fmt_for_avpvs
(reference lib/test_config.py:447-480, :172-180); CPVS formats from
Pvs.get_vcodec_and_pix_fmt_for_cpvs (:188-227).
"""
from dataclasses import dataclass

YUV420P, YUV422P, YUV444P, YUV420P10LE, YUV422P10LE, YUV444P10LE, UYVY422, V210 = range(8)

NAMES = {
    "yuv420p": YUV420P, "yuv422p": YUV422P, "yuv444p": YUV444P,
    "yuv420p10le": YUV420P10LE, "yuv422p10le": YUV422P10LE, "yuv444p10le": YUV444P10LE,
    "uyvy422": UYVY422, "v210": V210,
}
BY_ID = {v: k for k, v in NAMES.items()}


@dataclass(frozen=True)
class Fmt:
    id: int
    name: str
    depth: int
    hsub: int
    vsub: int
    packed: bool

    @property
    def bytes_per_sample(self):
        return 2 if self.depth > 8 else 1


def fmt(f):
    """Fmt for an id, an ffmpeg pix_fmt name or a Fmt."""
    if isinstance(f, Fmt):
        return f
    fid = NAMES[f] if isinstance(f, str) else int(f)
    name = BY_ID[fid]
    depth = 10 if fid in (YUV420P10LE, YUV422P10LE, YUV444P10LE, V210) else 8
    hsub = 0 if fid in (YUV444P, YUV444P10LE) else 1
    vsub = 1 if fid in (YUV420P, YUV420P10LE) else 0
    return Fmt(fid, name, depth, hsub, vsub, fid in (UYVY422, V210))


def v210_linesize(w):
    """libavcodec/v210enc.c: ((w + 47) / 48) * 48 * 8 / 3 bytes per line."""
    return ((w + 47) // 48) * 48 * 8 // 3


def plane_shapes(f, w, h):
    """[(rows, samples-or-bytes per row)] per plane."""
    f = fmt(f)
    if f.id == UYVY422:
        return [(h, 2 * w)]
    if f.id == V210:
        return [(h, v210_linesize(w))]
    cw, ch = -((-w) >> f.hsub), -((-h) >> f.vsub)
    return [(h, w), (ch, cw), (ch, cw)]


def frame_bytes(f, w, h):
    """Bytes of one dense frame (the SURVEY section 8 frame-size shorthand)."""
    f = fmt(f)
    if f.packed:
        r, c = plane_shapes(f, w, h)[0]
        return r * c
    return sum(r * c for r, c in plane_shapes(f, w, h)) * f.bytes_per_sample
