"""HIP pad / v210 / stall compositing vs the CPU restatement -- bit-exact.

pad: vf_pad (lib/ffmpeg.py:1183, :1209); v210: v210enc (lib/test_config.py:
208-215); stall: spec PP-STALL-1 (bufferer, p03_generateAvPvs.py:236-243,
parity unpinned against bufferer itself)."""
import os

import numpy as np
import pytest

import pyoracle as po
import synth

pytestmark = pytest.mark.gpu
GOLDEN_SPINNER = os.path.join(os.path.dirname(__file__), "golden", "spinner-128-white.png")


def _batch(fmt, frames, gpu, dense):
    """Frames as a pitched FrameBatch (16-B rows: the vector paths) or a dense
    frame-interleaved one (rows at any byte offset: the sample-by-sample paths)."""
    import torch
    from pixpath.frames import FrameBatch
    if not dense:
        return FrameBatch.from_numpy(fmt, synth.batch(frames), device=gpu)
    h, w = frames[0][0].shape
    b = FrameBatch.interleaved(fmt, w, h, len(frames), device=gpu)
    planes = synth.batch(frames)
    for p in range(3):
        b.planes[p].copy_(torch.from_numpy(np.ascontiguousarray(planes[p])).to(gpu))
    return b


@pytest.mark.parametrize("fmt,sw,sh,dw,dh", [
    (po.YUV420P, 1920, 800, 1920, 1080),       # SRC 3840x1600 -> AVPVS 1920x800, PC CPVS
    (po.YUV422P10LE, 1920, 1012, 1920, 1080),  # 4096x2160 SRC
    (po.YUV420P10LE, 1280, 533, 1280, 800),    # tablet, odd offset rounded to the chroma grid
    (po.YUV422P, 31, 17, 64, 40),
    (po.YUV422P10LE, 1280, 720, 1920, 1080),   # 16-B aligned shift: vector loads
    (po.YUV422P10LE, 1276, 700, 1920, 1080),   # ox = 322: unaligned shift
])
@pytest.mark.parametrize("dense", [False, True])
def test_pad_matches_oracle(gpu, fmt, sw, sh, dw, dh, dense):
    from pixpath import ops
    rng = np.random.default_rng(3)
    frames = [synth.noise_frame(rng, fmt, sw, sh) for _ in range(2)]
    src = _batch(fmt, frames, gpu, dense)
    out = ops.pad(src, dw, dh).to_numpy()
    for i in range(2):
        ref = po.pad(fmt, frames[i], dw, dh, (dw - sw) // 2, (dh - sh) // 2)
        for p in range(3):
            np.testing.assert_array_equal(out[p][i], ref[p])


@pytest.mark.parametrize("w,h", [(1920, 1080), (1280, 720), (100, 7), (52, 3), (8, 2), (10, 2)])
def test_v210_matches_oracle(gpu, w, h):
    from pixpath import ops
    from pixpath.frames import FrameBatch
    rng = np.random.default_rng(11)
    # full 10-bit range so the [4, 1019] clip is exercised
    frames = [[rng.integers(0, 1024, s).astype(np.uint16) for s in po.plane_shapes(po.YUV422P10LE, w, h)]
              for _ in range(2)]
    src = FrameBatch.from_numpy(po.YUV422P10LE, synth.batch(frames), device=gpu)
    out = ops.v210_pack(src).to_numpy()[0]
    for i in range(2):
        np.testing.assert_array_equal(out[i], po.v210_pack(frames[i]))


@pytest.mark.parametrize("fmt,w,h,dense", [
    (po.YUV420P, 1920, 1080, False), (po.YUV422P10LE, 1920, 1080, False), (po.YUV420P10LE, 1920, 1080, False),
    (po.YUV422P, 1920, 1080, False), (po.YUV420P, 202, 170, True), (po.YUV422P10LE, 330, 132, True),
])
def test_stall_compose_matches_oracle(gpu, fmt, w, h, dense):
    from pixpath import ops, spinner
    anim, _ = spinner.load_apng(GOLDEN_SPINNER)
    rng = np.random.default_rng(404)
    frames = [synth.noise_frame(rng, fmt, w, h) for _ in range(3)]
    src = _batch(fmt, frames, gpu, dense)
    ops.spinner_upload(anim, fmt)
    src_idx = np.array([2, 2, -1, 0, 1], np.int32)
    sp_idx = np.array([0, 5, 7, -1, 3], np.int32)
    out = ops.stall_compose(src, src_idx, sp_idx).to_numpy()
    depth = po.fmt_info(fmt)[0]
    for k in range(len(src_idx)):
        if src_idx[k] >= 0:
            base = frames[src_idx[k]]
        else:
            base = [np.full(s, (16 if p == 0 else 128) << (depth - 8), dtype=po.plane_dtype(fmt))
                    for p, s in enumerate(po.plane_shapes(fmt, w, h))]
        ref = base if sp_idx[k] < 0 else po.overlay_spinner(fmt, base, po.spinner_to_yuva(anim[sp_idx[k]], fmt))
        for p in range(3):
            np.testing.assert_array_equal(out[p][k], ref[p], err_msg="frame %d plane %d" % (k, p))


def test_stall_compose_long_runs_across_tiles(gpu):
    """A stall run as the product composes it (one frozen frame repeated,
    spinner animating) mixed with source changes and black frames, 300 frames:
    the kernel's tiles of G frames per wave (one source load, G stores), the
    256-frame launch split and a source change inside a tile all equal the
    oracle."""
    from pixpath import ops, spinner
    fmt, w, h = po.YUV422P10LE, 320, 180
    anim, _ = spinner.load_apng(GOLDEN_SPINNER)
    rng = np.random.default_rng(405)
    frames = [synth.noise_frame(rng, fmt, w, h) for _ in range(3)]
    src = _batch(fmt, frames, gpu, False)
    ops.spinner_upload(anim, fmt)
    src_idx = np.array([0] * 131 + [1] * 7 + [-1] * 5 + [2, 0, 2, 1] * 39 + [1], np.int32)
    sp_idx = (np.arange(len(src_idx)) % len(anim)).astype(np.int32)
    sp_idx[140:150] = -1
    out = ops.stall_compose(src, src_idx, sp_idx).to_numpy()
    depth = po.fmt_info(fmt)[0]
    for k in list(range(0, len(src_idx), 7)) + [130, 131, 137, 138, 142, 143, 255, 256, len(src_idx) - 1]:
        if src_idx[k] >= 0:
            base = frames[src_idx[k]]
        else:
            base = [np.full(s, (16 if p == 0 else 128) << (depth - 8), dtype=po.plane_dtype(fmt))
                    for p, s in enumerate(po.plane_shapes(fmt, w, h))]
        ref = base if sp_idx[k] < 0 else po.overlay_spinner(fmt, base, po.spinner_to_yuva(anim[sp_idx[k]], fmt))
        for p in range(3):
            np.testing.assert_array_equal(out[p][k], ref[p], err_msg="frame %d plane %d" % (k, p))


@pytest.mark.parametrize("fmt,w,h,W,H", [
    (po.YUV420P, 1920, 800, 1920, 1080), (po.YUV420P, 1920, 1080, 1920, 1080), (po.YUV422P, 1920, 1012, 1920, 1080),
    (po.YUV420P10LE, 1920, 1080, 1920, 1080), (po.YUV420P10LE, 1920, 800, 1920, 1080),
    (po.YUV422P10LE, 1920, 1080, 1920, 1080), (po.YUV422P10LE, 1280, 534, 1280, 720), (po.YUV420P10LE, 100, 38, 100, 50),
    (po.YUV420P, 102, 38, 102, 50), (po.YUV420P, 1280, 720, 1920, 1080), (po.YUV422P10LE, 1276, 716, 1920, 1080),
    (po.YUV420P10LE, 1276, 716, 1920, 1080),
])
@pytest.mark.parametrize("content", ["legal", "checker", "noise"])
def test_fused_cpvs_matches_chain(gpu, fmt, w, h, W, H, content):
    """pp_cpvs_execute == pad -> swscale (bicubic, -> uyvy422 / yuv422p10le) -> v210, bit-exact;
    legal-range noise, and full-range 0/max checkerboards and noise (the 4:2:0 ->
    4:2:2 vertical filter's clip and v210's [4, 1019] clip)."""
    from pixpath import ops
    from pixpath.frames import FrameBatch
    rng = np.random.default_rng(8)
    if content == "legal":
        frames = [synth.noise_frame(rng, fmt, w, h) for _ in range(2)]
    else:
        frames = [synth.extreme_frame(content, fmt, w, h, seed=i) for i in range(2)]
    src = FrameBatch.from_numpy(fmt, synth.batch(frames), device=gpu)
    out = ops.cpvs(src, W, H).to_numpy()[0]
    depth = po.fmt_info(fmt)[0]
    for i in range(2):
        padded = po.pad(fmt, frames[i], W, H, (W - w) // 2, (H - h) // 2)
        if depth == 8:
            (ref,) = po.scale(fmt, padded, po.UYVY422, W, H)
        else:
            p422 = padded if fmt == po.YUV422P10LE else po.scale(fmt, padded, po.YUV422P10LE, W, H)
            ref = po.v210_pack(p422)
        np.testing.assert_array_equal(out[i], ref)


@pytest.mark.parametrize("fmt,w,h,W,H", [
    (po.YUV420P, 102, 38, 102, 50), (po.YUV420P10LE, 100, 38, 100, 50), (po.YUV422P10LE, 330, 132, 336, 140),
    (po.YUV422P, 202, 100, 210, 104),
])
def test_fused_cpvs_dense_rows(gpu, fmt, w, h, W, H):
    """Source rows at arbitrary byte offsets (a dense frame-interleaved batch): the
    sample-by-sample staging path gives the same bytes as the oracle chain."""
    from pixpath import ops
    rng = np.random.default_rng(81)
    frames = [synth.noise_frame(rng, fmt, w, h) for _ in range(3)]
    out = ops.cpvs(_batch(fmt, frames, gpu, True), W, H).to_numpy()[0]
    depth = po.fmt_info(fmt)[0]
    for i in range(3):
        padded = po.pad(fmt, frames[i], W, H, (W - w) // 2, (H - h) // 2)
        if depth == 8:
            (ref,) = po.scale(fmt, padded, po.UYVY422, W, H)
        else:
            p422 = padded if fmt == po.YUV422P10LE else po.scale(fmt, padded, po.YUV422P10LE, W, H)
            ref = po.v210_pack(p422)
        np.testing.assert_array_equal(out[i], ref)
