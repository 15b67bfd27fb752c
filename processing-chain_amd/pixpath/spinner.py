"""Spinner animation loader (APNG -> RGBA8 frames).

The reference hands `-s util/spinner-128-white.png` (lib/parse_args.py:99,
default) to bufferer (p03_generateAvPvs.py:240).  That file is an 8-frame
128x128 RGBA APNG with 8/89 s per frame whose frames 2..8 are sub-rectangle
updates; this module composes them into full canvases (dispose/blend ops of
the APNG spec) so the GPU gets n full RGBA frames.  Pure Python + zlib: host
setup work, done once per run.
"""
import struct
import zlib

import numpy as np

_SIG = b"\x89PNG\r\n\x1a\n"


def _chunks(data):
    if data[:8] != _SIG:
        raise ValueError("not a PNG file")
    i = 8
    while i < len(data):
        (n,) = struct.unpack(">I", data[i:i + 4])
        typ = data[i + 4:i + 8]
        yield typ, data[i + 8:i + 8 + n]
        i += 12 + n


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    if pa <= pb and pa <= pc:
        return a
    return b if pb <= pc else c


def _unfilter(raw, w, h, bpp=4):
    stride = w * bpp
    out = np.zeros((h, stride), dtype=np.uint8)
    prev = bytearray(stride)
    pos = 0
    for y in range(h):
        ft = raw[pos]
        line = bytearray(raw[pos + 1:pos + 1 + stride])
        pos += 1 + stride
        if ft == 1:
            for x in range(bpp, stride):
                line[x] = (line[x] + line[x - bpp]) & 255
        elif ft == 2:
            for x in range(stride):
                line[x] = (line[x] + prev[x]) & 255
        elif ft == 3:
            for x in range(stride):
                left = line[x - bpp] if x >= bpp else 0
                line[x] = (line[x] + ((left + prev[x]) >> 1)) & 255
        elif ft == 4:
            for x in range(stride):
                left = line[x - bpp] if x >= bpp else 0
                ul = prev[x - bpp] if x >= bpp else 0
                line[x] = (line[x] + _paeth(left, prev[x], ul)) & 255
        elif ft != 0:
            raise ValueError("bad PNG filter %d" % ft)
        out[y] = np.frombuffer(bytes(line), dtype=np.uint8)
        prev = line
    return out.reshape(h, w, bpp)


def load_apng(src):
    """Return (frames [n, h, w, 4] uint8, delays [n] seconds) of an RGBA8 (A)PNG."""
    data = open(src, "rb").read() if isinstance(src, str) else bytes(src)
    ihdr = None
    frames_ctl = []  # (fcTL fields, [data...])
    default_data = []
    cur = None
    for typ, body in _chunks(data):
        if typ == b"IHDR":
            ihdr = struct.unpack(">IIBBBBB", body)
            if ihdr[2] != 8 or ihdr[3] != 6 or ihdr[6] != 0:
                raise ValueError("only non-interlaced 8-bit RGBA PNGs are supported")
        elif typ == b"fcTL":
            seq, fw, fh, fx, fy, dn, dd, dop, bop = struct.unpack(">IIIIIHHBB", body)
            cur = [(fw, fh, fx, fy, dn / (dd or 100), dop, bop), []]
            frames_ctl.append(cur)
        elif typ == b"IDAT":
            default_data.append(body)
            if cur is not None:
                cur[1].append(body)
        elif typ == b"fdAT":
            cur[1].append(body[4:])
    W, H = ihdr[0], ihdr[1]
    if not frames_ctl:  # plain PNG
        img = _unfilter(zlib.decompress(b"".join(default_data)), W, H)
        return img[None].copy(), np.array([0.0])
    canvas = np.zeros((H, W, 4), dtype=np.uint8)
    out, delays = [], []
    for (fw, fh, fx, fy, delay, dop, bop), parts in frames_ctl:
        sub = _unfilter(zlib.decompress(b"".join(parts)), fw, fh)
        saved = canvas.copy()
        region = canvas[fy:fy + fh, fx:fx + fw]
        if bop == 0:  # APNG_BLEND_OP_SOURCE
            region[...] = sub
        else:  # APNG_BLEND_OP_OVER (8-bit, straight alpha)
            a = sub[..., 3:4].astype(np.float64) / 255.0
            b = region[..., 3:4].astype(np.float64) / 255.0
            oa = a + b * (1 - a)
            rgb = np.where(oa > 0, (sub[..., :3] * a + region[..., :3] * b * (1 - a)) / np.maximum(oa, 1e-12), 0)
            region[..., :3] = np.round(rgb).astype(np.uint8)
            region[..., 3:4] = np.round(oa * 255).astype(np.uint8)
        out.append(canvas.copy())
        delays.append(delay)
        if dop == 1:  # APNG_DISPOSE_OP_BACKGROUND
            canvas[fy:fy + fh, fx:fx + fw] = 0
        elif dop == 2:  # APNG_DISPOSE_OP_PREVIOUS
            canvas = saved
    return np.stack(out), np.array(delays)
