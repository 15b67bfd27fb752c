"""Seeded synthetic frames: legal-range noise and smooth
moving content (zone plate + gradient + bars).  Legal ranges: 8-bit Y [16,235],
C [16,240]; 10-bit Y [64,940], C [64,960]."""
import numpy as np

import pyoracle as po


def legal(depth, chroma):
    s = 1 << (depth - 8)
    return (16 * s, (240 if chroma else 235) * s)


def noise_frame(rng, fmt, w, h):
    depth, hs, vs = po.fmt_info(fmt)
    dt = np.uint16 if depth > 8 else np.uint8
    out = []
    for p, (r, c) in enumerate(po.plane_shapes(fmt, w, h)):
        lo, hi = legal(depth, p > 0)
        out.append(rng.integers(lo, hi + 1, (r, c)).astype(dt))
    return out


def smooth_frame(t, fmt, w, h):
    """Moving zone plate + translating gradient + moving bars, frame index t."""
    depth, hs, vs = po.fmt_info(fmt)
    dt = np.uint16 if depth > 8 else np.uint8
    out = []
    for p, (r, c) in enumerate(po.plane_shapes(fmt, w, h)):
        lo, hi = legal(depth, p > 0)
        yy, xx = np.mgrid[0:r, 0:c].astype(np.float64)
        sx = xx * (w / c)
        sy = yy * (h / r)
        zp = np.cos(((sx - w / 2) ** 2 + (sy - h / 2) ** 2) * (np.pi / (4.0 * max(w, h))) + 0.3 * t)
        grad = ((sx + 7 * t) % w) / w
        bars = ((sy + 3 * t) // max(8, h // 16)) % 2
        v = 0.45 * (zp + 1) / 2 + 0.35 * grad + 0.2 * bars
        if p:
            v = 0.5 + 0.3 * (v - 0.5) * (1 if p == 1 else -1)
        out.append(np.clip(np.round(lo + v * (hi - lo)), lo, hi).astype(dt))
    return out


def batch(frames):
    """list of per-frame plane lists -> list of [N, r, c] stacks."""
    return [np.stack([f[p] for f in frames]) for p in range(len(frames[0]))]


def extreme_frame(kind, fmt, w, h, seed=0, seams_x=(), seams_y=()):
    """Full-range test patterns (values 0 and 2^depth - 1, beyond the legal
    range, as real decodes can carry): they drive swscale's 15-bit clip of the
    horizontal intermediates and the output clip to [0, max].
      checker   1-px checkerboard 0/max (the largest filter overshoot)
      checker4  4-px checkerboard
      steps     0/max step edges at the given source columns / rows (strip and
                segment seams), alternating
      noise     uniform noise over the full range [0, max]"""
    depth, hs, vs = po.fmt_info(fmt)
    dt = np.uint16 if depth > 8 else np.uint8
    mx = (1 << depth) - 1
    rng = np.random.default_rng(seed)
    out = []
    for p, (r, c) in enumerate(po.plane_shapes(fmt, w, h)):
        yy, xx = np.mgrid[0:r, 0:c]
        if kind == "checker":
            v = ((yy + xx + p) & 1) * mx
        elif kind == "checker4":
            v = (((yy >> 2) + (xx >> 2) + p) & 1) * mx
        elif kind == "steps":
            sx = np.searchsorted(np.asarray(sorted(int(x) >> (hs if p else 0) for x in seams_x)), xx, side="right")
            sy = np.searchsorted(np.asarray(sorted(int(y) >> (vs if p else 0) for y in seams_y)), yy, side="right")
            v = ((sx + sy + p) & 1) * mx
        elif kind == "noise":
            v = rng.integers(0, mx + 1, (r, c))
        else:
            raise ValueError(kind)
        out.append(v.astype(dt))
    return out
