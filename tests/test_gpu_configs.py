"""BASELINE configs 1 and 4 end to end through the GPU-backend commands
(pixpath.cli, what pixpath.ffmpeg's gpu builders run), with Y4M files standing
in for the ffmpeg decode/encode pipes (there is no ffmpeg on the box); EVERY
output frame is checked against the oracle chain.

Config 1 (P2SXM00 short test shape): one SRC
  3840x2160 yuv422p10le @60 -> SI/TI (analyse_src) -> p01 encode_segment's
  pixel work (encseg: scale=W:-2 to three quality levels) -> p03 short AVPVS
  (upscale to 1920x1080 yuv422p10le, bicubic) for 3 HRCs, one with a stall ->
  p04 PC CPVS (v210).  Per-frame shapes are the real ones; the clip is 0.5 s
  (30 frames) instead of P2SXM00's 10 s to keep the test's disk use small.
Config 4 (long test with stalls): 3 segments x 2 s @60 (960x540 yuv422p10le
  quality level) -> create_avpvs_segment each (scale into the overlay's
  yuv420p, -pix_fmt yuv422p10le, 1920x1080 canvas of D*R frames) -> concat ->
  stalls [[2,1.5],[4,1.0]] with util/spinner-128-white.png -> PC CPVS (v210).
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import pyoracle as po
import synth
from pixpath import chain, io as pio

pytestmark = pytest.mark.gpu
GOLDEN_SPINNER = os.path.join(os.path.dirname(__file__), "golden", "spinner-128-white.png")
POOL = ThreadPoolExecutor(16)  # the oracle's C calls release the GIL


def _write_y4m(path, fmt_name, frames, w, h, rate=60):
    wr = pio.Y4MWriter(path, fmt_name, w, h, rate)
    for f in frames:
        wr.write(pio.join_planes(synth.batch([f])))
    wr.close()


def _frames_of(path, batch=32):
    """Yield (index, [planes]) of every frame of a Y4M file."""
    r = pio.open_reader(path)
    k = 0
    for b in r.batches(batch):
        for i in range(b[0].shape[0]):
            yield k, [p[i] for p in b]
            k += 1
    r.close()


def _check_stream(path, expected_fn, n_expected):
    """Compare every frame of `path` with expected_fn(k) (computed in parallel)."""
    n = 0
    pending = []
    for k, got in _frames_of(path):
        pending.append((k, got, POOL.submit(expected_fn, k)))
        if len(pending) >= 32:
            for kk, g, fut in pending:
                _eq(g, fut.result(), kk)
            pending = []
        n += 1
    for kk, g, fut in pending:
        _eq(g, fut.result(), kk)
    assert n == n_expected


def _eq(got, ref, k):
    for p in range(len(ref)):
        if not np.array_equal(got[p], ref[p]):
            bad = np.argwhere(got[p] != ref[p])
            pytest.fail("frame %d plane %d: %d mismatches, first at %s" % (k, p, len(bad), tuple(bad[0])))


def _v210_check(path, frames_fn, n):
    raw = np.memmap(path, np.uint8, mode="r")
    fb = po.v210_linesize(1920) * 1080
    assert raw.size == n * fb

    def one(k):
        ref = po.v210_pack(frames_fn(k))
        return np.array_equal(np.asarray(raw[k * fb:(k + 1) * fb]).reshape(ref.shape), ref)
    assert all(POOL.map(one, range(n)))


def _stall_ref(frames_fn, anim, seq, fmt):
    yuva = {}

    def ref(k):
        s, sp = seq[k]
        base = frames_fn(s)
        if sp < 0:
            return base
        if sp not in yuva:
            yuva[sp] = po.spinner_to_yuva(anim[sp], fmt)
        return po.overlay_spinner(fmt, base, yuva[sp])
    return ref


def test_config1_short_test_chain(gpu, tmp_path):
    import siti_ref
    from pixpath import cli, siti, spinner
    n = 30
    src_frames = [synth.smooth_frame(t, po.YUV422P10LE, 3840, 2160) for t in range(n)]
    src = str(tmp_path / "P2SXM00_SRC001.y4m")
    _write_y4m(src, "yuv422p10le", src_frames, 3840, 2160)
    # SI/TI hook (analyse_src; the ffprobe keys are given: no ffprobe on the box)
    yp = siti.analyse_src(src, 0, src_info={"r_frame_rate": "60", "width": 3840, "height": 2160},
                          stream_sizes={"v": os.path.getsize(src), "a": 0})
    import yaml
    d = yaml.safe_load(open(yp))
    rsi, rti = siti_ref.siti(np.stack([f[0] for f in src_frames]))
    np.testing.assert_allclose(d["siti"]["si_frames"], rsi, rtol=1e-4)
    np.testing.assert_allclose(d["siti"]["ti_frames"][1:], rti[1:], rtol=1e-9)
    anim, delays = spinner.load_apng(GOLDEN_SPINNER)
    for hrc, (qw, stall) in enumerate([(1920, None), (1280, "[[0.2,0.1]]"), (960, None)]):
        qh = chain.scale_height_keep_aspect(3840, 2160, qw)
        seg = str(tmp_path / ("seg%d.y4m" % hrc))
        assert cli.main(["encseg", "--input", src, "--start", "0", "--duration", "0.5", "--width", str(qw),
                         "--pix-fmt", "yuv422p10le", "--select", "", "--fps", "60", "--in-fps", "60", seg]) == 0

        def seg_ref(k, qw=qw, qh=qh):
            return po.scale(po.YUV422P10LE, src_frames[k], po.YUV422P10LE, qw, qh, po.SWS_BICUBIC)
        _check_stream(seg, seg_ref, n)
        avpvs = str(tmp_path / ("avpvs%d.y4m" % hrc))
        assert cli.main(["avpvs", "-y", "--input", seg, "--size", "1920x1080", "--flags", "bicubic",
                         "--pix-fmt", "yuv422p10le", avpvs]) == 0
        cache = {}

        def av_ref(k, seg_ref=seg_ref, qw=qw, qh=qh):
            if k not in cache:
                cache[k] = po.scale(po.YUV422P10LE, seg_ref(k), po.YUV422P10LE, 1920, 1080, po.SWS_BICUBIC)
            return cache[k]
        _check_stream(avpvs, av_ref, n)
        final, count, frame_fn = avpvs, n, av_ref
        if stall:
            final = str(tmp_path / ("pvs%d.y4m" % hrc))
            assert cli.main(["stall", "-y", "--input", avpvs, "--buffer", stall, "--spinner", GOLDEN_SPINNER,
                             "--black-frame", final]) == 0
            seq = cli.stall_schedule([[0.2, 0.1]], 60, n, False, delays)
            frame_fn = _stall_ref(av_ref, anim, seq, po.YUV422P10LE)
            count = len(seq)
            _check_stream(final, frame_fn, count)
        cpvs = str(tmp_path / ("cpvs%d.raw" % hrc))
        assert cli.main(["cpvs", "-y", "--input", final, "--fps", "60", "--vcodec", "v210", "--pix-fmt",
                         "yuv422p10le", cpvs]) == 0
        _v210_check(cpvs, frame_fn, count)
        for p in (seg, avpvs, final, cpvs):
            if os.path.exists(p):
                os.remove(p)


def test_config4_long_test_chain(gpu, tmp_path):
    from pixpath import cli, spinner
    rate, seg_s, n_seg = 60, 2, 3
    per = seg_s * rate
    rng = np.random.default_rng(404)
    segs = [[synth.noise_frame(rng, po.YUV422P10LE, 960, 540) for _ in range(per)] for _ in range(n_seg)]
    tmp_avis = []
    for i, frames in enumerate(segs):
        s = str(tmp_path / ("seg%d.y4m" % i))
        _write_y4m(s, "yuv422p10le", frames, 960, 540)
        t = str(tmp_path / ("tmp_seg%d.y4m" % i))
        assert cli.main(["avpvs", "-y", "--input", s, "--size", "1920x1080", "--pix-fmt", "yuv422p10le",
                         "--fps", "60", "--duration", str(seg_s), "--overlay-yuv420", t]) == 0
        os.remove(s)
        tmp_avis.append(t)
    # create_avpvs_long_concat: stream copy of the segment AVPVSes (here: frames in order)
    concat = str(tmp_path / "PVS_concat_wo_buffer.y4m")
    wr = pio.Y4MWriter(concat, "yuv422p10le", 1920, 1080, rate)
    for t in tmp_avis:
        for b in pio.open_reader(t).batches(32):
            wr.write(pio.join_planes(b))
        os.remove(t)
    wr.close()

    def concat_ref(k):
        f = segs[k // per][k % per]
        mid = po.scale(po.YUV422P10LE, f, po.YUV420P, 1920, 1080, po.SWS_BICUBIC)
        return po.scale(po.YUV420P, mid, po.YUV422P10LE, 1920, 1080, po.SWS_BICUBIC)
    events = [[2, 1.5], [4, 1.0]]
    final = str(tmp_path / "PVS.y4m")
    assert cli.main(["stall", "-y", "--input", concat, "--buffer", "[[2,1.5],[4,1.0]]", "--spinner", GOLDEN_SPINNER,
                     "--black-frame", final]) == 0
    os.remove(concat)
    anim, delays = spinner.load_apng(GOLDEN_SPINNER)
    seq = cli.stall_schedule(events, rate, n_seg * per, False, delays)
    assert len(seq) == 360 + 90 + 60
    ref = _stall_ref(concat_ref, anim, seq, po.YUV422P10LE)
    _check_stream(final, ref, len(seq))
    cpvs = str(tmp_path / "PVS_PC.raw")
    assert cli.main(["cpvs", "-y", "--input", final, "--fps", "60", "--vcodec", "v210", "--pix-fmt", "yuv422p10le",
                     cpvs]) == 0
    os.remove(final)
    _v210_check(cpvs, ref, len(seq))


def test_config4_long_test_through_gpu_ffv1(gpu, tmp_path):
    """Config 4 with the gpu backend's default AVPVS codec (FFV1 on the GPU,
    pixpath AVIs): create_avpvs_segment -> GPU-FFV1 canvases, the concat is a
    packet copy (`cli concat`), the bufferer step works at the packet level
    (pass-through frames copied, only the stall frames composed and encoded),
    and the PC CPVS decodes on the GPU.  Every v210 frame equals the oracle's
    two-stage chain + PP-STALL-1 + v210; the pass-through packets of the
    stalled AVPVS are the concat's packets byte for byte: after the segment
    encode no frame is decoded and re-encoded except the stalls' sources."""
    from pixpath import avi, cli, spinner
    rate, seg_s, n_seg = 60, 2, 3
    per = seg_s * rate
    rng = np.random.default_rng(404)
    segs = [[synth.noise_frame(rng, po.YUV422P10LE, 960, 540) for _ in range(per)] for _ in range(n_seg)]
    lst = str(tmp_path / "PVS_tmp_filelist.txt")
    with open(lst, "w") as fl:
        for i, frames in enumerate(segs):
            s = str(tmp_path / ("seg%d.y4m" % i))
            _write_y4m(s, "yuv422p10le", frames, 960, 540)
            t = str(tmp_path / ("tmp_seg%d.avi" % i))
            assert cli.main(["avpvs", "-y", "--input", s, "--size", "1920x1080", "--pix-fmt", "yuv422p10le",
                             "--fps", "60", "--duration", str(seg_s), "--overlay-yuv420", "--aopts=-an",
                             "--gpu-ffv1", t]) == 0
            os.remove(s)
            fl.write("file %s\n" % t)
    concat = str(tmp_path / "PVS_concat_wo_buffer.avi")
    assert cli.main(["concat", "-y", "--filelist", lst, "--duration", str(n_seg * seg_s), concat]) == 0
    final = str(tmp_path / "PVS.avi")
    assert cli.main(["stall", "-y", "--input", concat, "--buffer", "[[2,1.5],[4,1.0]]", "--spinner", GOLDEN_SPINNER,
                     "--black-frame", "--aopts=-an", "--gpu-ffv1", final]) == 0
    anim, delays = spinner.load_apng(GOLDEN_SPINNER)
    seq = cli.stall_schedule([[2, 1.5], [4, 1.0]], rate, n_seg * per, False, delays)
    _, pc = avi.read_packets(concat)
    _, pf = avi.read_packets(final)
    assert len(pc) == n_seg * per and len(pf) == len(seq)
    assert all(pf[k] == pc[s] for k, (s, sp) in enumerate(seq) if sp < 0)
    cpvs = str(tmp_path / "PVS_PC.raw")
    assert cli.main(["cpvs", "-y", "--input", final, "--fps", "60", "--vcodec", "v210", "--pix-fmt", "yuv422p10le",
                     "--gpu-ffv1", cpvs]) == 0

    def concat_ref(k):
        f = segs[k // per][k % per]
        mid = po.scale(po.YUV422P10LE, f, po.YUV420P, 1920, 1080, po.SWS_BICUBIC)
        return po.scale(po.YUV420P, mid, po.YUV422P10LE, 1920, 1080, po.SWS_BICUBIC)
    _v210_check(cpvs, _stall_ref(concat_ref, anim, seq, po.YUV422P10LE), len(seq))
