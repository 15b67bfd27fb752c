"""Scaler over whole 600-frame batches of DISTINCT frames, and full-range
extreme patterns (VERDICT r1 "what's weak").

* 600 distinct seeded frames in HBM (generated on the GPU per frame, seeded),
  the first, the last and 12 spread frames of the output checked against the
  oracle, for the config-2 plans (lanczos and bicubic upscale) and the
  config-3 plans (2160p -> 1080p, 10-bit and 8-bit sources).  A kernel that
  read or wrote frame f' for frame f fails here.
* 0/max checkerboards and step edges placed at the output strip seams
  (multiples of 256 columns) and the segment seams of the plan, plus
  full-range noise: swscale's 15-bit intermediate clip (hScale*To15) and the
  output clip to [0, 2^d - 1] are driven on purpose.  Both scaler kernels.
"""
import numpy as np
import pytest

import pyoracle as po
import synth

pytestmark = pytest.mark.gpu

LONG_PLANS = [
    (po.YUV422P10LE, 1280, 720, po.YUV422P10LE, 1920, 1080, po.SWS_LANCZOS),   # config 2
    (po.YUV422P10LE, 1280, 720, po.YUV422P10LE, 1920, 1080, po.SWS_BICUBIC),   # config 2, reference filter
    (po.YUV422P10LE, 3840, 2160, po.YUV422P10LE, 1920, 1080, po.SWS_BICUBIC),  # config 3, 10-bit source
    (po.YUV420P, 3840, 2160, po.YUV422P10LE, 1920, 1080, po.SWS_BICUBIC),      # config 3, 8-bit source
]
FLAGS = {po.SWS_LANCZOS: "lanczos", po.SWS_BICUBIC: "bicubic", po.SWS_BILINEAR: "bilinear"}


def _ids(c):
    return "%dx%d_f%d->%dx%d_f%d_%s" % (c[1], c[2], c[0], c[4], c[5], c[3], FLAGS[c[6]])


@pytest.mark.parametrize("plan", LONG_PLANS, ids=_ids)
def test_600_distinct_frames(gpu, plan):
    import torch
    from pixpath import ops
    from pixpath.frames import FrameBatch
    sf, sw, sh, df, dw, dh, flags = plan
    n = 600
    src = FrameBatch(sf, sw, sh, n, device=gpu)
    depth = po.fmt_info(sf)[0]
    g = torch.Generator(device=gpu)
    g.manual_seed(600)
    for p in range(3):
        v = src.view(p)  # full-range noise, different in every frame
        v.copy_(torch.randint(0, 1 << depth, v.shape, generator=g, device=gpu, dtype=torch.int32).to(v.dtype))
    sc = ops.Scaler(sf, sw, sh, df, dw, dh, flags=FLAGS[flags])
    dst = sc(src)
    torch.cuda.synchronize()
    check = sorted({0, n - 1} | set(np.linspace(1, n - 2, 12).astype(int).tolist()))
    for f in check:
        frame = [src.view(p)[f].cpu().numpy() for p in range(3)]
        ref = po.scale(sf, frame, df, dw, dh, flags)
        for p in range(3):
            got = dst.view(p)[f].cpu().numpy()
            if not np.array_equal(got, ref[p]):
                bad = np.argwhere(got != ref[p])
                pytest.fail("frame %d plane %d: %d mismatches, first at %s" % (f, p, len(bad), tuple(bad[0])))
    # consecutive outputs differ (the inputs do): no frame was written twice
    for f in check[:-1]:
        assert not torch.equal(dst.view(0)[f], dst.view(0)[f + 1])


EXTREME_PLANS = LONG_PLANS + [
    (po.YUV420P10LE, 960, 540, po.YUV420P, 1920, 1080, po.SWS_BICUBIC),        # a3 overlay yuv420 (dither)
    (po.YUV420P, 1920, 1080, po.YUV422P10LE, 1920, 1080, po.SWS_BICUBIC),      # a3 / a5 -pix_fmt stages
    (po.YUV420P, 1280, 720, po.YUV420P, 1920, 1080, po.SWS_BICUBIC),
    (po.YUV422P10LE, 3840, 2160, po.YUV422P10LE, 960, 540, po.SWS_LANCZOS),    # long filters
]


@pytest.mark.parametrize("kernel", ["auto", "generic"])
@pytest.mark.parametrize("kind", ["checker", "checker4", "steps", "noise"])
@pytest.mark.parametrize("plan", EXTREME_PLANS, ids=_ids)
def test_full_range_extremes(gpu, plan, kind, kernel, monkeypatch):
    import torch
    from pixpath import ops
    from pixpath.frames import FrameBatch
    sf, sw, sh, df, dw, dh, flags = plan
    # output strip seams (256 columns) and segment seams (540 rows) mapped to source coordinates
    seams_x = [x * sw // dw for x in range(256, dw, 256)] + [x * sw // dw + 1 for x in range(256, dw, 256)]
    seams_y = [y * sh // dh for y in range(270, dh, 270)]
    frames = [synth.extreme_frame(kind, sf, sw, sh, seed=i, seams_x=seams_x, seams_y=seams_y) for i in range(2)]
    src = FrameBatch.from_numpy(sf, synth.batch(frames), device=gpu)
    out = ops.Scaler(sf, sw, sh, df, dw, dh, flags=FLAGS[flags], generic=kernel == "generic")(src).to_numpy()
    torch.cuda.synchronize()
    mx = (1 << po.fmt_info(df)[0]) - 1 if df not in (po.UYVY422, po.V210) else 255
    hit_clip = False
    for i in range(2):
        ref = po.scale(sf, frames[i], df, dw, dh, flags)
        for p, r in enumerate(ref):
            hit_clip |= bool((r == 0).any() or (r == mx).any())
            if not np.array_equal(out[p][i], r):
                bad = np.argwhere(out[p][i] != r)
                pytest.fail("frame %d plane %d: %d mismatches, first at %s got %d want %d" % (
                    i, p, len(bad), tuple(bad[0]), out[p][i][tuple(bad[0])], r[tuple(bad[0])]))
    if kind == "steps" or (kind == "checker" and dw >= sw):  # a downscale averages a 1-px checker to grey
        assert hit_clip, "pattern did not reach the output clip"
