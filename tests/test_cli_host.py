"""Host-side pieces of the GPU pipeline (CPU): Y4M/raw I/O, stall schedule
(PP-STALL-1), fps duplication counts == the vf_fps map."""
import os

import numpy as np
import pytest

import pyoracle as po
import synth
from pixpath import chain, io as pio
from pixpath.cli import _fps_counts, stall_schedule


def test_y4m_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    frames = [synth.noise_frame(rng, po.YUV422P10LE, 48, 20) for _ in range(3)]
    raw = pio.join_planes(synth.batch(frames))
    p = str(tmp_path / "a.y4m")
    w = pio.Y4MWriter(p, "yuv422p10le", 48, 20, "60000/1001")
    w.write(raw)
    w.close()
    r = pio.open_reader(p)
    assert (r.w, r.h, r.fmt.name, r.rate) == (48, 20, "yuv422p10le", pio.Fraction(60000, 1001))
    got = list(r.batches(2))
    assert [g[0].shape[0] for g in got] == [2, 1]
    back = [np.concatenate([g[i] for g in got]) for i in range(3)]
    for a, b in zip(back, synth.batch(frames)):
        np.testing.assert_array_equal(a, b)
    assert pio.probe(p)["stream"]["pix_fmt"] == "yuv422p10le"


def test_split_join_planes():
    rng = np.random.default_rng(1)
    fr = synth.batch([synth.noise_frame(rng, po.YUV420P, 30, 14) for _ in range(2)])
    raw = pio.join_planes(fr)
    for a, b in zip(pio.split_planes(raw, "yuv420p", 30, 14), fr):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("a,b,n", [(30, 60, 17), (24, 60, 33), (60, 30, 20), (60, 60, 9), (25, 60, 50),
                                   ("30000/1001", 60, 31)])
def test_fps_counts_match_map(a, b, n):
    counts = _fps_counts(a, b)
    m = chain.fps_index_map(n, a, b)
    expanded = [i for i in range(n) for _ in range(counts(i))]
    assert expanded == m


def test_stall_schedule_spinner():
    # AVPVS 6 s @ 10 fps, stalls [[2, 1.5], [4, 1.0]] (media time), spinner 8 x 0.25 s
    seq = stall_schedule([[2, 1.5], [4, 1.0]], 10, 60, False, [0.25] * 8)
    assert len(seq) == 60 + 15 + 10
    assert seq[:20] == [(i, -1) for i in range(20)]
    stall1 = seq[20:35]
    assert all(s == 19 for s, _ in stall1)
    assert [sp for _, sp in stall1] == [0, 0, 0, 1, 1, 2, 2, 2, 3, 3, 4, 4, 4, 5, 5]
    assert seq[35:55] == [(i, -1) for i in range(20, 40)]
    assert all(s == 39 and sp >= 0 for s, sp in seq[55:65])
    assert seq[65:] == [(i, -1) for i in range(40, 60)]


def test_stall_at_zero_is_black():
    seq = stall_schedule([[0, 0.5]], 10, 4, False, [0.1] * 8, black_frame=True)
    assert seq[:5] == [(-1, k) for k in range(5)] and seq[5:] == [(i, -1) for i in range(4)]
    seq = stall_schedule([[0, 0.5]], 10, 4, False, [0.1] * 8, black_frame=False)
    assert seq[0] == (0, 0)


def test_freeze_with_skipping_keeps_length():
    seq = stall_schedule([[1, 0.5], [3, 0.2]], 10, 50, True)
    assert len(seq) == 50
    assert seq[10:15] == [(9, -1)] * 5 and seq[15] == (15, -1)
    assert seq[30:32] == [(29, -1)] * 2


def test_gpu_avpvs_short_composes_stalls_in_the_same_pass(monkeypatch):
    """gpu backend: create_avpvs_short of a PVS with stalls also writes the
    stalled AVPVS (--stall-output), with the bufferer step's own arguments."""
    import types
    from pixpath import ffmpeg as pff
    monkeypatch.setenv("PIXPATH_SPINNER", "/opt/spinner.png")
    monkeypatch.setattr(pff, "_backend", "gpu")
    pp = types.SimpleNamespace(coding_width=1920, coding_height=1080)
    ql = types.SimpleNamespace(width=1280, height=720)
    seg = types.SimpleNamespace(quality_level=ql, get_segment_file_path=lambda: "/db/seg0.mkv")
    pvs = types.SimpleNamespace(
        test_config=types.SimpleNamespace(post_processings=[pp]), has_buffering=lambda: True,
        has_framefreeze=lambda: False, get_avpvs_wo_buffer_file_path=lambda: "/db/avpvs/P_wo.avi",
        get_avpvs_file_path=lambda: "/db/avpvs/P.avi", segments=[seg], get_pix_fmt_for_avpvs=lambda: "yuv422p10le",
        src=types.SimpleNamespace(stream_info={"coded_width": 3840, "coded_height": 2160}),
        get_buff_events_media_time=lambda: [[4, 1.5], [8, 1.0]])
    cmd = pff.create_avpvs_short(pvs, overwrite=True)
    assert "--stall-output /db/avpvs/P.avi --buffer '[[4,1.5],[8,1.0]]' --black-frame --spinner /opt/spinner.png" in cmd
    assert cmd.endswith("/db/avpvs/P_wo.avi")
    monkeypatch.delenv("PIXPATH_SPINNER")
    monkeypatch.setattr(pff, "default_spinner_path", lambda: None)
    assert "--stall-output" not in pff.create_avpvs_short(pvs, overwrite=True)


def test_gpu_ffv1_opt_in_flags(monkeypatch):
    """PIXPATH_FFV1=gpu: AVPVS writers encode FFV1 on the GPU, AVPVS readers decode it there."""
    from pixpath import ffmpeg as pff
    monkeypatch.setenv("PIXPATH_FFV1", "gpu")
    monkeypatch.delenv("PIXPATH_FFV1_SLICES", raising=False)
    a = pff._gpu_cli("avpvs", ["-y", "--vopts", pff.FFV1_OPTS, "/o.avi"])
    assert a.endswith("--gpu-ffv1 --ffv1-slices 8x8 /o.avi")
    monkeypatch.setenv("PIXPATH_FFV1_SLICES", "16x16")
    assert pff._gpu_cli("avpvs", ["-y", "--vopts", pff.FFV1_OPTS, "/o.avi"]).endswith("--ffv1-slices 16x16 /o.avi")
    monkeypatch.delenv("PIXPATH_FFV1_SLICES")
    assert pff._gpu_cli("avpvs", ["-y", "--vopts", "-c:v libx264", "/o.mp4"]).endswith("--ffv1-input /o.mp4")
    assert pff._gpu_cli("cpvs", ["-y", "/c.avi"]).endswith("--gpu-ffv1 /c.avi")
    assert pff._gpu_cli("stall", ["-y", "/s.avi"]).endswith("--gpu-ffv1 /s.avi")
    monkeypatch.delenv("PIXPATH_FFV1")  # the default: FFV1 on the GPU
    assert pff._gpu_cli("cpvs", ["-y", "/c.avi"]).endswith("--gpu-ffv1 /c.avi")
    monkeypatch.setenv("PIXPATH_FFV1", "ffmpeg")
    assert "--gpu-ffv1" not in pff._gpu_cli("cpvs", ["-y", "/c.avi"])


def test_cli_concat_copies_packets_and_cuts(tmp_path):
    """`cli concat` (gpu backend's create_avpvs_long_concat for GPU-FFV1
    segment AVIs): packets of the listed AVIs in order, cut at
    round(duration * rate) frames like `-t`, same configuration record."""
    from fractions import Fraction
    from pixpath import avi, cli
    rng = np.random.default_rng(5)
    extra = b"cfg-record"
    files, allp = [], []
    for k in range(3):
        p = str(tmp_path / ("tmp_seg%d.avi" % k))
        w = avi.AviWriter(p, 64, 36, 60, extradata=extra)
        for _ in range(120):
            pk = rng.integers(0, 256, int(rng.integers(5, 300)), dtype=np.uint8).tobytes()
            w.write_packet(pk)
            allp.append(pk)
        w.close()
        files.append(p)
    lst = str(tmp_path / "list.txt")
    with open(lst, "w") as f:
        f.writelines("file %s\n" % p for p in files)
    out = str(tmp_path / "concat.avi")
    assert cli.main(["concat", "-y", "--filelist", lst, "--duration", "5", out]) == 0
    info, got = avi.read_packets(out)
    assert got == allp[:300] and info["extradata"] == extra and info["rate"] == Fraction(60)
    assert cli.main(["concat", "-y", "--filelist", lst, out]) == 0
    assert avi.read_packets(out)[1] == allp
    bad = str(tmp_path / "bad.avi")
    w = avi.AviWriter(bad, 64, 36, 60, extradata=b"other")
    w.write_packet(b"x")
    w.close()
    with open(lst, "a") as f:
        f.write("file %s\n" % bad)
    with pytest.raises(SystemExit):
        cli.main(["concat", "-y", "--filelist", lst, out])


def test_gpu_backend_long_concat_string(tmp_path, monkeypatch):
    """gpu backend + GPU FFV1: create_avpvs_long_concat writes the reference's
    filelist and returns `pixpath.cli concat` with the same -t total."""
    import shlex
    import ref_stubs
    from test_host_reference_parity import Methods
    from pixpath import ffmpeg as pff
    sc = {"type": "long", "src": [3840, 2160], "segments": [[1280, 720, 2], [1280, 720, 3]],
          "pps": [["pc", 1920, 1080]], "target_pix_fmt": "yuv422p10le",
          "events": [["quality_level", 2], ["quality_level", 3]], "pvs_id": "P2LXM00_SRC001_HRC001"}
    tc, pvs, _ = ref_stubs.build(sc, str(tmp_path), Methods)
    os.makedirs(os.path.join(str(tmp_path), "avpvs"), exist_ok=True)
    tc.root = str(tmp_path)
    pff.set_backend("gpu")
    try:
        got = pff.create_avpvs_long_concat(pvs, overwrite=True)
    finally:
        pff.set_backend("ffmpeg")
    a = shlex.split(got)
    i = a.index("concat")
    assert a[i + 1] == "-y" and a[a.index("--filelist") + 1] == pvs.get_avpvs_file_list()
    assert a[a.index("--duration") + 1] == "5" and a[-1] == pvs.get_tmp_wo_audio_path()
    assert open(pvs.get_avpvs_file_list()).read().count("file ") == 2
    monkeypatch.setenv("PIXPATH_FFV1", "ffmpeg")
    pff.set_backend("gpu")
    try:
        assert pff.create_avpvs_long_concat(pvs, overwrite=True).startswith("ffmpeg -nostdin -y -f concat")
    finally:
        pff.set_backend("ffmpeg")


def test_interleaved_batch_on_a_storage_slice():
    """FrameBatch.interleaved over rows k.. of another batch's storage views
    those frames (as_strided's offset is absolute: the slice's own offset
    must be kept) -- the FFV1 reader hands out such views."""
    import torch
    from pixpath.frames import FrameBatch
    b = FrameBatch.interleaved("yuv422p10le", 16, 6, 4, device="cpu")
    b.storage.copy_((torch.arange(b.storage.numel()) % 251).view_as(b.storage).to(torch.uint8))
    for k in range(4):
        v = FrameBatch.interleaved("yuv422p10le", 16, 6, 4 - k, device="cpu", storage=b.storage[k:])
        for p in range(3):
            assert torch.equal(v.view(p)[0], b.view(p)[k])


def test_ffv1_writer_slice_grid_setting(monkeypatch):
    """PIXPATH_FFV1_SLICES picks the AVPVS writers' FFV1 slice grid (default 8x8)."""
    from pixpath import ffv1
    monkeypatch.delenv("PIXPATH_FFV1_SLICES", raising=False)
    assert ffv1.default_slices() == (8, 8)
    monkeypatch.setenv("PIXPATH_FFV1_SLICES", "16x16")
    assert ffv1.default_slices() == (16, 16)
    for bad in ("16", "0x4", "ax4"):
        monkeypatch.setenv("PIXPATH_FFV1_SLICES", bad)
        with pytest.raises(ValueError):
            ffv1.default_slices()


def test_pixpath_ffv1_detection_and_reader_fallback(tmp_path, monkeypatch):
    """is_pixpath_ffv1 (the packet-level stall's test) holds only for records
    exactly pixpath's encoder's; the GPU decoder (open_avpvs_reader) also
    takes FFmpeg's `-coder 1 -context 1` records (gpu_decodable); a corrupt
    record or another codec falls back to ffmpeg's decoder through
    pixpath.io."""
    import ffv1_ref as ref
    from pixpath import avi, ffv1, io as pio
    gen = ref.gen_extradata(ref.make_prof(10, 1, 0, 2, 2, ref.ffmpeg_context1_sets(10)))
    assert not ffv1.is_pixpath_ffv1({"fourcc": b"FFV1", "w": 640, "h": 360, "extradata": gen})
    assert ffv1.gpu_decodable({"fourcc": b"FFV1", "w": 640, "h": 360, "extradata": gen})
    assert not ffv1.gpu_decodable({"fourcc": b"FFV1", "w": 640, "h": 360, "extradata": gen[:-1] + b"\0"})
    rec = ffv1.Ffv1Encoder("yuv422p10le", 640, 360, slices=(4, 4), host_only=True).extradata
    base = {"fourcc": b"FFV1", "w": 640, "h": 360}
    assert ffv1.is_pixpath_ffv1(dict(base, extradata=rec))
    assert not ffv1.is_pixpath_ffv1(dict(base, extradata=rec[:-1] + bytes([rec[-1] ^ 1])))  # CRC
    assert not ffv1.is_pixpath_ffv1(dict(base, extradata=b"\x00" * 40))
    assert not ffv1.is_pixpath_ffv1(dict(base, fourcc=b"H264", extradata=rec))
    other = ffv1.Ffv1Encoder("yuv422p10le", 640, 360, slices=(2, 2), host_only=True).extradata
    assert ffv1.is_pixpath_ffv1(dict(base, extradata=other))  # its own grid: still pixpath's
    path = str(tmp_path / "ffmpeg_ffv1.avi")
    w = avi.AviWriter(path, 640, 360, 60, extradata=b"not-pixpath-record")
    w.write_packet(b"\x00" * 16)
    w.close()
    sentinel = object()
    monkeypatch.setattr(pio, "open_reader", lambda p, **k: sentinel)
    assert ffv1.open_avpvs_reader(path) is sentinel
    assert ffv1.open_avpvs_reader(str(tmp_path / "x.y4m")) is sentinel


def test_codec_provenance_in_the_p03_log_line(monkeypatch):
    """p03 logs every builder string as an `ffmpegCommand:` line
    (p03_generateAvPvs.py:41-59).  With the GPU FFV1 (default) the line names
    the codec and slice grid; with PIXPATH_FFV1=ffmpeg it carries the
    reference's own FFV1 options (the reference-faithful bitstream)."""
    from pixpath import ffmpeg as pff
    from p03_log import p03_log_line
    args = ["-y", "--input", "/db/videoSegments/seg.mkv", "--size", "1920x1080", "--pix-fmt", "yuv422p10le",
            "--vopts", pff.FFV1_OPTS, "--aopts", "-c:a flac", "/db/avpvs/P.avi"]
    monkeypatch.delenv("PIXPATH_FFV1", raising=False)
    monkeypatch.setenv("PIXPATH_FFV1_SLICES", "16x16")
    line = p03_log_line(pff._collapse(pff._gpu_cli("avpvs", args)), "/db/videoSegments", "/db/srcVid")
    assert line.startswith("ffmpegCommand: ") and "--gpu-ffv1 --ffv1-slices 16x16" in line
    assert "seg.mkv" in line and "/db/videoSegments/" not in line
    monkeypatch.setenv("PIXPATH_FFV1", "ffmpeg")
    line = p03_log_line(pff._collapse(pff._gpu_cli("avpvs", args)), "/db/videoSegments", "/db/srcVid")
    assert "--gpu-ffv1" not in line and "-coder 1 -context 1 -slicecrc 1" in line


def test_decoder_route_by_stream_shape(monkeypatch):
    """decoder_route (open_avpvs_reader's choice, VERDICT r5 item 3 / ADVICE r5):
    pixpath's intra FFV1 goes to the GPU; an FFmpeg-made GOP stream (the
    reference's AVPVS: 200 serial chains per 600 frames, slower on the GPU
    than on the host) goes to ffmpeg when ffmpeg exists, else to the GPU;
    PIXPATH_FFV1_DECODE forces either; PIXPATH_FFV1=ffmpeg sends records not
    written by pixpath to ffmpeg; a record the GPU decoder refuses goes to
    ffmpeg."""
    import ffv1_ref as ref
    from pixpath import ffv1
    monkeypatch.delenv("PIXPATH_FFV1_DECODE", raising=False)
    monkeypatch.delenv("PIXPATH_FFV1", raising=False)
    base = {"fourcc": b"FFV1", "w": 640, "h": 360}
    own = dict(base, extradata=ffv1.Ffv1Encoder("yuv422p10le", 640, 360, slices=(8, 8), host_only=True).extradata)
    gops = dict(base, extradata=ref.gen_extradata(ref.make_prof(10, 1, 0, 2, 2, ref.ffmpeg_context1_sets(10),
                                                                tidx=(1, 1), coder=2, gop=12)))
    bad = dict(base, extradata=gops["extradata"][:-1] + b"\0")
    for have in (True, False):
        assert ffv1.decoder_route(own, have_ffmpeg=have) == "gpu"
        assert ffv1.decoder_route(bad, have_ffmpeg=have) == "ffmpeg"
    assert ffv1.decoder_route(gops, have_ffmpeg=True) == "ffmpeg"
    assert ffv1.decoder_route(gops, have_ffmpeg=False) == "gpu"
    monkeypatch.setenv("PIXPATH_FFV1_DECODE", "gpu")
    assert ffv1.decoder_route(gops, have_ffmpeg=True) == "gpu"
    assert ffv1.decoder_route(bad, have_ffmpeg=True) == "ffmpeg"
    monkeypatch.setenv("PIXPATH_FFV1_DECODE", "ffmpeg")
    assert ffv1.decoder_route(own, have_ffmpeg=False) == "ffmpeg"
    monkeypatch.delenv("PIXPATH_FFV1_DECODE")
    monkeypatch.setenv("PIXPATH_FFV1", "ffmpeg")
    assert ffv1.decoder_route(gops, have_ffmpeg=False) == "ffmpeg"
    assert ffv1.decoder_route(own, have_ffmpeg=False) == "gpu"


def test_writer_split_by_open_writers(monkeypatch):
    """writer_split (the AVPVS writer's encoder lanes): default_split() lanes
    for a writer coding alone on its device, one encoder when other writers
    are open there; PIXPATH_FFV1_SPLIT forces the count for every writer and
    is range-checked."""
    from pixpath import ffv1
    monkeypatch.delenv("PIXPATH_FFV1_SPLIT", raising=False)
    assert ffv1.writer_split(0, opened=0) == 2
    assert ffv1.writer_split(0, opened=3) == 1
    monkeypatch.setenv("PIXPATH_FFV1_SPLIT", "3")
    assert ffv1.writer_split(0, opened=0) == 3 and ffv1.writer_split(0, opened=2) == 3
    monkeypatch.setenv("PIXPATH_FFV1_SPLIT", "9")
    with pytest.raises(ValueError):
        ffv1.writer_split(0, opened=0)
