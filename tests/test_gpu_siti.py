"""HIP P.910 SI/TI vs the numpy reference (oracle/siti_ref.py) -- 1e-4 relative.

Tolerance (north_star): SI/TI within 1e-4 relative of the numpy reference.
The kernel's TI moments are exact integers, so TI is compared at 1e-12."""
import numpy as np
import pytest

import siti_ref
import synth
import pyoracle as po

pytestmark = pytest.mark.gpu
RTOL_SI = 1e-4


def _run(frames, depth, gpu, prev=None, normalize=False):
    import torch
    from pixpath import ops
    dt = torch.uint16 if depth > 8 else torch.uint8
    t = torch.from_numpy(np.ascontiguousarray(frames.astype(np.uint16 if depth > 8 else np.uint8))).to(gpu)
    pt = None
    if prev is not None:
        pt = torch.from_numpy(np.ascontiguousarray(prev.astype(np.uint16 if depth > 8 else np.uint8))).to(gpu)
    assert t.dtype == dt
    si, ti = ops.siti(t, depth, prev=pt, normalize=normalize)
    torch.cuda.synchronize()
    return si.cpu().numpy(), ti.cpu().numpy()


@pytest.mark.parametrize("depth,w,h,content", [
    (8, 1920, 1080, "smooth"), (10, 1920, 1080, "smooth"), (8, 1920, 1080, "noise"),
    (10, 3840, 2160, "smooth"), (8, 333, 97, "noise"), (10, 2050, 33, "noise"), (8, 3, 3, "noise"),
])
def test_siti_matches_numpy(gpu, depth, w, h, content):
    fmt = po.YUV420P10LE if depth > 8 else po.YUV420P
    rng = np.random.default_rng(910)
    n = 4
    if content == "smooth":
        frames = np.stack([synth.smooth_frame(t, fmt, w, h)[0] for t in range(n)])
    else:
        frames = np.stack([synth.noise_frame(rng, fmt, w, h)[0] for _ in range(n)])
    si, ti = _run(frames, depth, gpu)
    rsi, rti = siti_ref.siti(frames)
    np.testing.assert_allclose(si, rsi, rtol=RTOL_SI, atol=1e-9)
    assert np.isnan(ti[0]) and np.isnan(rti[0])
    np.testing.assert_allclose(ti[1:], rti[1:], rtol=1e-12, atol=1e-12)


def test_siti_known_answers(gpu):
    # constant frames: SI = TI = 0; a static repeated frame: TI = 0
    c = np.full((3, 64, 80), 100, np.uint8)
    si, ti = _run(c, 8, gpu)
    assert np.all(si == 0) and np.all(ti[1:] == 0)
    # vertical edge: step of 100 at column 40 -> Sobel |Gx| = 400 on two columns
    e = np.zeros((2, 32, 80), np.uint8)
    e[:, :, 40:] = 100
    si, _ = _run(e, 8, gpu)
    rsi, _ = siti_ref.siti(e)
    np.testing.assert_allclose(si, rsi, rtol=1e-12)
    # global brightness step of +5 between frames: TI = 0 (std of a constant)
    g = np.stack([np.full((16, 16), 50, np.uint8), np.full((16, 16), 55, np.uint8)])
    _, ti = _run(g, 8, gpu)
    assert ti[1] == 0


def test_siti_prev_halo_equals_single_pass(gpu):
    """Frame-range sharding with a 1-frame halo reproduces the single pass."""
    frames = np.stack([synth.smooth_frame(t, po.YUV420P10LE, 640, 360)[0] for t in range(9)])
    si, ti = _run(frames, 10, gpu)
    si_a, ti_a = _run(frames[:4], 10, gpu)
    si_b, ti_b = _run(frames[4:], 10, gpu, prev=frames[3])
    np.testing.assert_array_equal(np.concatenate([si_a, si_b]), si)
    np.testing.assert_array_equal(np.concatenate([ti_a, ti_b])[1:], ti[1:])


def test_siti_config2_length(gpu):
    """600 frames (config 2 length) against the C oracle on every 50th frame."""
    frames = np.stack([synth.smooth_frame(t % 37, po.YUV420P10LE, 1920, 1080)[0] for t in range(600)])
    si, ti = _run(frames, 10, gpu)
    idx = np.arange(1, 600, 50)
    for i in idx:
        rsi = siti_ref.si_frame(frames[i])
        rti = siti_ref.ti_frame(frames[i], frames[i - 1])
        assert abs(si[i] - rsi) <= RTOL_SI * abs(rsi)
        assert abs(ti[i] - rti) <= 1e-12 * max(1.0, abs(rti))


@pytest.mark.parametrize("depth,w", [(10, 1984), (10, 1985), (8, 497), (8, 496), (10, 3969)])
def test_siti_tile_and_wave_boundaries(gpu, depth, w):
    """Widths around the 496-px wave span and the 1984-px workgroup span."""
    fmt = po.YUV420P10LE if depth > 8 else po.YUV420P
    rng = np.random.default_rng(w)
    frames = np.stack([synth.noise_frame(rng, fmt, w, 37)[0] for _ in range(3)])
    si, ti = _run(frames, depth, gpu)
    rsi, rti = siti_ref.siti(frames)
    np.testing.assert_allclose(si, rsi, rtol=RTOL_SI, atol=1e-9)
    np.testing.assert_allclose(ti[1:], rti[1:], rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("depth", [8, 10])
def test_siti_unaligned_pitched_view(gpu, depth):
    """A pitched view starting one sample into each row takes the unaligned path."""
    import torch
    from pixpath import ops
    fmt = po.YUV420P10LE if depth > 8 else po.YUV420P
    rng = np.random.default_rng(5)
    w, h, n = 643, 41, 5
    frames = np.stack([synth.noise_frame(rng, fmt, w, h)[0] for _ in range(n)])
    dt = np.uint16 if depth > 8 else np.uint8
    big = np.zeros((n, h, w + 5), dt)
    big[:, :, 1:w + 1] = frames
    t = torch.from_numpy(big).to(gpu)[:, :, 1:w + 1]
    si, ti = ops.siti(t, depth)
    torch.cuda.synchronize()
    rsi, rti = siti_ref.siti(frames)
    np.testing.assert_allclose(si.cpu().numpy(), rsi, rtol=RTOL_SI, atol=1e-9)
    np.testing.assert_allclose(ti.cpu().numpy()[1:], rti[1:], rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("depth,w", [(8, 333), (10, 1366)])
def test_siti_padded_pitch(gpu, depth, w):
    """Aligned pitched rows wider than the frame (vector path, partial last granule)."""
    import torch
    from pixpath import ops
    fmt = po.YUV420P10LE if depth > 8 else po.YUV420P
    rng = np.random.default_rng(w)
    h, n = 45, 4
    frames = np.stack([synth.noise_frame(rng, fmt, w, h)[0] for _ in range(n)])
    dt = np.uint16 if depth > 8 else np.uint8
    pitch = (w + 63) // 64 * 64
    big = np.full((n, h, pitch), 7, dt)
    big[:, :, :w] = frames
    t = torch.from_numpy(big).to(gpu)[:, :, :w]
    si, ti = ops.siti(t, depth)
    torch.cuda.synchronize()
    rsi, rti = siti_ref.siti(frames)
    np.testing.assert_allclose(si.cpu().numpy(), rsi, rtol=RTOL_SI, atol=1e-9)
    np.testing.assert_allclose(ti.cpu().numpy()[1:], rti[1:], rtol=1e-12, atol=1e-12)


def test_siti_normalize_8bit_equals_shifted_10bit(gpu):
    """KAT of PP_SITI_NORMALIZE: an 8-bit clip and the same
    clip << 2 at 10 bits give equal SI/TI on the 8-bit scale (a power-of-two
    scaling: exact), and the 10-bit raw values are 4x the 8-bit ones."""
    rng = np.random.default_rng(88)
    f8 = np.stack([synth.smooth_frame(t, po.YUV420P, 1920, 1080)[0] for t in range(3)] +
                  [synth.noise_frame(rng, po.YUV420P, 1920, 1080)[0]])
    f10 = f8.astype(np.uint16) << 2
    si8, ti8 = _run(f8, 8, gpu, normalize=True)
    si10, ti10 = _run(f10, 10, gpu, normalize=True)
    np.testing.assert_array_equal(si8, si10)
    np.testing.assert_array_equal(ti8[1:], ti10[1:])
    raw10, rawt10 = _run(f10, 10, gpu)
    np.testing.assert_array_equal(raw10, 4 * si8)
    np.testing.assert_array_equal(rawt10[1:], 4 * ti8[1:])
    rsi, rti = siti_ref.siti(f10, bitdepth=10, normalize=True)
    np.testing.assert_allclose(si10, rsi, rtol=RTOL_SI)
    np.testing.assert_allclose(ti10[1:], rti[1:], rtol=1e-12)


@pytest.mark.parametrize("fmt_name,batch", [("yuv422p10le", 16), ("yuv420p", 7)])
def test_siti_of_file_streamed_luma_only(gpu, tmp_path, fmt_name, batch):
    """SRC-analysis path: a Y4M read luma-only (chroma skipped) through the
    pinned double-buffered stream, batches smaller than the clip so the TI
    halo crosses batch boundaries; equals the numpy reference per frame."""
    from pixpath import io as pio, siti
    fmt = {"yuv422p10le": po.YUV422P10LE, "yuv420p": po.YUV420P}[fmt_name]
    n, w, h = 40, 640, 360
    frames = [synth.smooth_frame(t, fmt, w, h) for t in range(n)]
    path = str(tmp_path / "src.y4m")
    wr = pio.Y4MWriter(path, fmt_name, w, h, 60)
    for f in frames:
        wr.write(pio.join_planes(synth.batch([f])))
    wr.close()
    luma = np.stack([f[0] for f in frames])
    depth = 10 if "10" in fmt_name else 8
    si, ti, d = siti.siti_of_file(path, batch=batch, with_depth=True)
    assert d == depth and len(si) == n
    rsi, rti = siti_ref.siti(luma)
    np.testing.assert_allclose(si, rsi, rtol=RTOL_SI, atol=1e-9)
    assert np.isnan(ti[0])
    np.testing.assert_allclose(ti[1:], rti[1:], rtol=1e-12, atol=1e-12)
    sin, tin = siti.siti_of_file(path, batch=batch, normalize=True)
    np.testing.assert_array_equal(sin, si / (1 << (depth - 8)))
