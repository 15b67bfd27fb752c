"""create_avpvs_segment's two-stage conversion as ONE plan (row a3, VERDICT r1
item 9): `scale=W:H:flags=bicubic` into the overlay's yuv420p, then
libavfilter's yuv420p -> -pix_fmt conversion (bicubic, same size)
(lib/ffmpeg.py:1037-1048) -- pp_scale_chain_plan_create.

Every output plane is bit-exact with the oracle's two stages run one after the
other (po.scale twice), for the fused one-launch path (kernel_path > 0: both
stages inside strip_kernel, the 4:2:0 -> 4:2:2 chroma filter fed from an LDS
ring) and for the two-launch fallback (first stages that are not strip plans).
Distinct full-range frames, dithered 10-bit sources, ragged sizes, and a
600-frame config-4-shaped batch with first/last/spread frames checked.
"""
import numpy as np
import pytest

import pyoracle as po
import synth

pytestmark = pytest.mark.gpu

FLAGS = {po.SWS_LANCZOS: "lanczos", po.SWS_BICUBIC: "bicubic"}
CASES = [
    # src fmt, sw, sh, target, dw, dh, flags
    (po.YUV420P10LE, 1280, 720, po.YUV422P10LE, 1920, 1080, po.SWS_BICUBIC),   # config 4 (dithered first stage)
    (po.YUV422P10LE, 1280, 720, po.YUV422P10LE, 1920, 1080, po.SWS_BICUBIC),
    (po.YUV420P, 1280, 720, po.YUV422P10LE, 1920, 1080, po.SWS_BICUBIC),
    (po.YUV420P, 1280, 720, po.YUV422P, 1920, 1080, po.SWS_BICUBIC),
    (po.YUV420P10LE, 1280, 720, po.YUV420P10LE, 1920, 1080, po.SWS_BICUBIC),
    (po.YUV422P10LE, 3840, 2160, po.YUV422P10LE, 1920, 1080, po.SWS_BICUBIC),  # downscaled long-test SRC
    (po.YUV420P, 960, 540, po.YUV422P10LE, 1920, 800, po.SWS_BICUBIC),         # letterboxed canvas
    (po.YUV420P10LE, 1000, 562, po.YUV422P10LE, 1366, 770, po.SWS_BICUBIC),    # ragged strips
    (po.YUV420P, 1920, 1080, po.YUV422P10LE, 1920, 1080, po.SWS_BICUBIC),      # unscaled first stage: 2 launches
    (po.YUV422P, 640, 360, po.YUV420P, 1280, 720, po.SWS_BICUBIC),             # yuv420p target: one stage
]


def _ids(c):
    return "%dx%d_f%d->%dx%d_f%d" % (c[1], c[2], c[0], c[4], c[5], c[3])


def _oracle(sf, frame, df, dw, dh, flags):
    mid = po.scale(sf, frame, po.YUV420P, dw, dh, flags)
    return mid if df == po.YUV420P else po.scale(po.YUV420P, mid, df, dw, dh, po.SWS_BICUBIC)


def _run(gpu, case, frames):
    from pixpath import ops
    from pixpath.frames import FrameBatch
    sf, sw, sh, df, dw, dh, flags = case
    names = {v: k for k, v in po.FMT_BY_NAME.items()}
    src = FrameBatch.from_numpy(names[sf], [np.stack([f[p] for f in frames]) for p in range(3)], device=gpu)
    sc = ops.Scaler(names[sf], sw, sh, names[df], dw, dh, flags=FLAGS[flags], chain=True)
    return sc, sc(src).to_numpy()


@pytest.mark.parametrize("case", CASES, ids=_ids)
def test_chain_matches_two_stage_oracle(gpu, case):
    sf, sw, sh, df, dw, dh, flags = case
    rng = np.random.default_rng(sw + dh)
    frames = [synth.noise_frame(rng, sf, sw, sh) for _ in range(2)] + \
             [synth.extreme_frame(kind, sf, sw, sh, seed=3, seams_x=range(170, sw, 171), seams_y=range(90, sh, 91))
              for kind in ("checker", "steps", "noise")]
    sc, out = _run(gpu, case, frames)
    if case[:3] == (po.YUV420P, 1920, 1080):
        assert sc.kernel_path == 0   # the first stage is an unscaled converter
    elif df != po.YUV420P:
        assert sc.kernel_path > 0    # one launch
    for f, frame in enumerate(frames):
        ref = _oracle(sf, frame, df, dw, dh, flags)
        for p in range(3):
            if not np.array_equal(out[p][f], ref[p]):
                bad = np.argwhere(out[p][f] != ref[p])
                pytest.fail("frame %d plane %d: %d mismatches, first at %s" % (f, p, len(bad), tuple(bad[0])))


def test_chain_600_distinct_frames(gpu):
    """Config-4 canvas shape over a whole 600-frame batch: no frame mixed up."""
    import torch
    from pixpath import ops
    from pixpath.frames import FrameBatch
    sf, sw, sh, df, dw, dh = po.YUV420P10LE, 1280, 720, po.YUV422P10LE, 1920, 1080
    n = 600
    src = FrameBatch("yuv420p10le", sw, sh, n, device=gpu)
    g = torch.Generator(device=gpu)
    g.manual_seed(404)
    for p in range(3):
        v = src.view(p)
        v.copy_(torch.randint(0, 1024, v.shape, generator=g, device=gpu, dtype=torch.int32).to(v.dtype))
    sc = ops.Scaler("yuv420p10le", sw, sh, "yuv422p10le", dw, dh, flags="bicubic", chain=True)
    assert sc.kernel_path > 0
    dst = sc(src)
    torch.cuda.synchronize()
    for f in sorted({0, n - 1} | set(np.linspace(1, n - 2, 12).astype(int).tolist())):
        ref = _oracle(sf, [src.view(p)[f].cpu().numpy() for p in range(3)], df, dw, dh, po.SWS_BICUBIC)
        for p in range(3):
            assert np.array_equal(dst.view(p)[f].cpu().numpy(), ref[p]), "frame %d plane %d" % (f, p)
