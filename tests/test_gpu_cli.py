"""End-to-end GPU-backend commands (pixpath.cli, what pixpath.ffmpeg's gpu
builders run) through the pinned double-buffered pipeline, with Y4M/raw files
standing in for the ffmpeg decode/encode pipes (no ffmpeg on the box).
Outputs are compared frame by frame with the oracle."""
import os

import numpy as np
import pytest

import pyoracle as po
import synth
from pixpath import chain, io as pio

pytestmark = pytest.mark.gpu
GOLDEN_SPINNER = os.path.join(os.path.dirname(__file__), "golden", "spinner-128-white.png")


def _write_y4m(path, fmt_name, frames, w, h, rate=60):
    wr = pio.Y4MWriter(path, fmt_name, w, h, rate)
    wr.write(pio.join_planes(synth.batch(frames)))
    wr.close()


def _read(path):
    r = pio.open_reader(path)
    planes = [np.concatenate(x) for x in zip(*r.batches(64))]
    r.close()
    return planes


def test_cli_avpvs_short_with_fps(gpu, tmp_path):
    """create_avpvs_short (gpu backend) incl. -f60: 30 fps 640x360 yuv420p -> 1280x720 @60."""
    from pixpath import cli
    rng = np.random.default_rng(1)
    frames = [synth.noise_frame(rng, po.YUV420P, 640, 360) for _ in range(37)]  # > one pipeline batch
    src, out = str(tmp_path / "seg.y4m"), str(tmp_path / "avpvs.y4m")
    _write_y4m(src, "yuv420p", frames, 640, 360, rate=30)
    assert cli.main(["avpvs", "-y", "--input", src, "--size", "1280x720", "--pix-fmt", "yuv420p", "--fps", "60",
                     "--batch", "16", out]) == 0
    got = _read(out)
    m = chain.fps_index_map(37, 30, 60)
    assert got[0].shape[0] == len(m) == 74
    for j in (0, 1, 2, 33, 73):
        ref = po.scale(po.YUV420P, frames[m[j]], po.YUV420P, 1280, 720, po.SWS_BICUBIC)
        for p in range(3):
            np.testing.assert_array_equal(got[p][j], ref[p])
    # overwrite convention: existing output and no -y -> untouched
    mtime = os.path.getmtime(out)
    assert cli.main(["avpvs", "--input", src, "--size", "1280x720", "--pix-fmt", "yuv420p", out]) == 0
    assert os.path.getmtime(out) == mtime


def test_cli_mobile_cpvs_scale(gpu, tmp_path):
    """create_cpvs mobile branch (gpu backend): `scale=1280:720:flags=bicubic` into
    x264's yuv420p as ONE swscale context (resize + 10->8-bit 4:2:2->4:2:0 with
    ffmpeg's ordered dither) -- what `cli avpvs --pix-fmt yuv420p` runs."""
    from pixpath import cli
    rng = np.random.default_rng(5)
    frames = [synth.noise_frame(rng, po.YUV422P10LE, 1920, 1080) for _ in range(5)]
    src, out = str(tmp_path / "avpvs.y4m"), str(tmp_path / "mobile.y4m")
    _write_y4m(src, "yuv422p10le", frames, 1920, 1080)
    assert cli.main(["avpvs", "-y", "--input", src, "--size", "1280x720", "--flags", "bicubic", "--pix-fmt",
                     "yuv420p", out]) == 0
    got = _read(out)
    assert got[0].shape == (5, 720, 1280)
    for j in range(5):
        ref = po.scale(po.YUV422P10LE, frames[j], po.YUV420P, 1280, 720, po.SWS_BICUBIC)
        for p in range(3):
            np.testing.assert_array_equal(got[p][j], ref[p])


def test_cli_avpvs_segment_canvas(gpu, tmp_path):
    """create_avpvs_segment: scale to the overlay's yuv420p, then -pix_fmt yuv422p10le, canvas of D*R frames
    with the last frame repeated (overlay eof_action=repeat)."""
    from pixpath import cli
    rng = np.random.default_rng(2)
    frames = [synth.noise_frame(rng, po.YUV420P10LE, 320, 180) for _ in range(50)]  # 50 frames @60 < 1 s
    src, out = str(tmp_path / "seg.y4m"), str(tmp_path / "tmp_seg.y4m")
    _write_y4m(src, "yuv420p10le", frames, 320, 180, rate=60)
    assert cli.main(["avpvs", "-y", "--input", src, "--size", "640x360", "--pix-fmt", "yuv422p10le", "--fps", "60",
                     "--duration", "1", "--overlay-yuv420", out]) == 0
    got = _read(out)
    assert got[0].shape[0] == 60
    for j in (0, 49, 59):
        mid = po.scale(po.YUV420P10LE, frames[min(j, 49)], po.YUV420P, 640, 360, po.SWS_BICUBIC)
        ref = po.scale(po.YUV420P, mid, po.YUV422P10LE, 640, 360, po.SWS_BICUBIC)
        for p in range(3):
            np.testing.assert_array_equal(got[p][j], ref[p])


@pytest.mark.parametrize("fmt,vcodec,pix", [("yuv420p", "rawvideo", "uyvy422"), ("yuv420p10le", "v210", "yuv422p10le"),
                                            ("yuv422p10le", "v210", "yuv422p10le"), ("yuv422p", "rawvideo", "uyvy422")])
def test_cli_cpvs_pad_pack(gpu, tmp_path, fmt, vcodec, pix):
    """create_cpvs PC: fps=60, pad 1920x800 -> 1920x1080, uyvy422 / v210."""
    from pixpath import cli
    fid = po.FMT_BY_NAME[fmt]
    rng = np.random.default_rng(3)
    frames = [synth.noise_frame(rng, fid, 1920, 800) for _ in range(3)]
    src, out = str(tmp_path / "avpvs.y4m"), str(tmp_path / "cpvs.raw")
    _write_y4m(src, fmt, frames, 1920, 800, rate=60)
    assert cli.main(["cpvs", "-y", "--input", src, "--fps", "60", "--vcodec", vcodec, "--pix-fmt", pix,
                     "--pad", "1920x1080", out]) == 0
    raw = np.fromfile(out, np.uint8)
    for i in range(3):
        padded = po.pad(fid, frames[i], 1920, 1080, 0, 140)
        if vcodec == "v210":
            p422 = padded if fid == po.YUV422P10LE else po.scale(fid, padded, po.YUV422P10LE, 1920, 1080)
            ref = po.v210_pack(p422)
        else:
            (ref,) = po.scale(fid, padded, po.UYVY422, 1920, 1080)
        fb = ref.size
        np.testing.assert_array_equal(raw[i * fb:(i + 1) * fb].reshape(ref.shape), ref)


def test_cli_stall_spinner(gpu, tmp_path):
    """bufferer replacement: stalls [[0.1, 0.1], [0.3, 0.05]] in a 0.5 s 1080p yuv422p10le AVPVS @60."""
    from pixpath import cli, spinner
    rng = np.random.default_rng(4)
    frames = [synth.noise_frame(rng, po.YUV422P10LE, 1920, 1080) for _ in range(30)]
    src, out = str(tmp_path / "wo_buffer.y4m"), str(tmp_path / "pvs.y4m")
    _write_y4m(src, "yuv422p10le", frames, 1920, 1080, rate=60)
    assert cli.main(["stall", "-y", "--input", src, "--buffer", "[[0.1,0.1],[0.3,0.05]]", "--spinner",
                     GOLDEN_SPINNER, "--black-frame", out]) == 0
    got = _read(out)
    anim, delays = spinner.load_apng(GOLDEN_SPINNER)
    seq = cli.stall_schedule([[0.1, 0.1], [0.3, 0.05]], 60, 30, False, delays)
    assert got[0].shape[0] == len(seq) == 30 + 6 + 3
    for k, (s, sp) in enumerate(seq):
        base = frames[s]
        ref = base if sp < 0 else po.overlay_spinner(po.YUV422P10LE, base, po.spinner_to_yuva(anim[sp], po.YUV422P10LE))
        for p in range(3):
            np.testing.assert_array_equal(got[p][k], ref[p], err_msg="frame %d" % k)


def test_cli_siti(gpu, tmp_path, capsys):
    import json
    import siti_ref
    from pixpath import cli
    frames = [synth.smooth_frame(t, po.YUV420P10LE, 1920, 1080) for t in range(12)]
    src = str(tmp_path / "src.y4m")
    _write_y4m(src, "yuv420p10le", frames, 1920, 1080)
    assert cli.main(["siti", "--input", src, "--batch", "5", "--per-frame"]) == 0
    res = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    rsi, rti = siti_ref.siti(np.stack([f[0] for f in frames]))
    np.testing.assert_allclose(res["si_frames"], rsi, rtol=1e-4)
    np.testing.assert_allclose(res["ti_frames"][1:], rti[1:], rtol=1e-9)
    assert res["ti_frames"][0] is None and abs(res["si"] - rsi.max()) <= 1e-4 * rsi.max()


@pytest.mark.parametrize("in_fps,out_fps,n,start,dur", [
    (60, 30, 40, "0.1", "0.5"),      # mod(n+1,2)
    (24, 15, 40, "0.25", "1.25"),    # the 62.5 % select pattern
    (60, 60, 20, "0", "0.2"),        # no select: fps=fps=orig
])
def test_cli_encseg_trim_scale_select_fps(gpu, tmp_path, in_fps, out_fps, n, start, dur):
    """p01 encode_segment, gpu backend (pixpath.cli encseg): -ss/-t trim, scale=W:-2:flags=bicubic
    (+ -pix_fmt yuv420p) on the GPU, select + fps on the host; every output frame vs the oracle."""
    from fractions import Fraction

    from pixpath import cli
    rng = np.random.default_rng(3)
    frames = [synth.noise_frame(rng, po.YUV422P10LE, 384, 216) for _ in range(n)]
    src, out = str(tmp_path / "src.y4m"), str(tmp_path / "enc.y4m")
    _write_y4m(src, "yuv422p10le", frames, 384, 216, rate=in_fps)
    sel = chain.select_expression(float(in_fps), float(out_fps)) if in_fps != out_fps else ""
    assert cli.main(["encseg", "--input", src, "--start", start, "--duration", dur, "--width", "256",
                     "--pix-fmt", "yuv420p", "--select", sel, "--fps", str(out_fps), "--in-fps", str(in_fps),
                     "--batch", "8", out]) == 0
    got = _read(out)
    h = chain.scale_height_keep_aspect(384, 216, 256)
    skip = int(round(Fraction(start) * in_fps))
    n_in = int(round(Fraction(dur) * in_fps))
    m = chain.select_fps_map(n_in, in_fps, out_fps, sel)
    assert got[0].shape == (len(m), h, 256)
    for j, k in enumerate(m):
        ref = po.scale(po.YUV422P10LE, frames[skip + k], po.YUV420P, 256, h, po.SWS_BICUBIC)
        for p in range(3):
            np.testing.assert_array_equal(got[p][j], ref[p], err_msg="out %d <- in %d plane %d" % (j, skip + k, p))


@pytest.mark.parametrize("mode", ["spinner", "skipping"])
def test_cli_avpvs_with_fused_stall(gpu, tmp_path, mode):
    """Section 8f-3: create_avpvs_short of a PVS with stalls composes the
    stalled AVPVS in the same pass (`cli avpvs --stall-output`).  Its output
    equals what the bufferer step (`cli stall`) makes from the written AVPVS;
    that step then keeps it (no second decode); with other arguments it
    regenerates."""
    import os
    from pixpath import cli
    rng = np.random.default_rng(8)
    frames = [synth.noise_frame(rng, po.YUV420P10LE, 320, 180) for _ in range(40)]
    src = str(tmp_path / "seg.y4m")
    _write_y4m(src, "yuv420p10le", frames, 320, 180, rate=60)
    wo, fused, plain = (str(tmp_path / n) for n in ("wo_buffer.y4m", "pvs.y4m", "plain.y4m"))
    buf = "[[0.1,0.1],[0.5,0.05]]" if mode == "spinner" else "[[0.1,0.1],[0.3,0.05]]"
    extra = ["--spinner", GOLDEN_SPINNER] if mode == "spinner" else ["--skipping"]
    assert cli.main(["avpvs", "-y", "--input", src, "--size", "640x360", "--pix-fmt", "yuv422p10le",
                     "--batch", "16", "--stall-output", fused, "--buffer", buf, "--black-frame"] + extra + [wo]) == 0
    assert os.path.isfile(fused + ".pixpath-stall.json")
    stall_args = ["--input", wo, "--buffer", buf, "--pix-fmt", "yuv422p10le", "--black-frame", "--vopts", "-c:v ffv1",
                  "--aopts", "-c:a pcm_s16le"] + extra
    assert cli.main(["stall", "-y"] + stall_args + [plain]) == 0
    assert open(fused, "rb").read() == open(plain, "rb").read()
    before = os.stat(fused).st_mtime_ns
    assert cli.main(["stall", "-y"] + stall_args + [fused]) == 0  # kept
    assert os.stat(fused).st_mtime_ns == before
    other = stall_args[:]
    other[other.index(buf)] = "[[0.2,0.1]]"
    assert cli.main(["stall", "-n"] + other + [fused]) == 0       # speculative output replaced
    assert cli.main(["stall", "-y"] + other + [plain]) == 0
    assert open(fused, "rb").read() == open(plain, "rb").read()
