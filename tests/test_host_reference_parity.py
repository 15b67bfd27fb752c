"""Host logic of the pixel path vs the reference's own outputs (CPU).

tests/golden/reference_fixtures.json was produced by running the reference's
Python (tests/golden/gen_reference_fixtures.py) on tests/scenarios.py; here
pixpath's restatements run on the same scenarios and must reproduce every
output byte for byte (ffmpeg backend) -- SURVEY.md section 8a rows a1-a10, a14."""
import json
import os
import types

import pytest

import ref_stubs
import scenarios
from pixpath import chain
from pixpath import ffmpeg as pff

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "reference_fixtures.json")
FX = json.load(open(GOLDEN))


class Methods:
    get_pix_fmt_for_avpvs = staticmethod(chain.get_pix_fmt_for_avpvs)
    get_vcodec_and_pix_fmt_for_cpvs = staticmethod(chain.get_vcodec_and_pix_fmt_for_cpvs)
    get_buff_events_media_time = staticmethod(chain.get_buff_events_media_time)
    hrc_get_buff_events_media_time = staticmethod(chain.hrc_get_buff_events_media_time)


def _call(fn, *a, **k):
    try:
        return fn(*a, **k)
    except SystemExit as e:
        return {"sys_exit": e.code}
    except Exception as e:
        return {"error": type(e).__name__}


@pytest.mark.parametrize("args,want", FX["avpvs_dims"])
def test_avpvs_dims(args, want):
    assert chain.calculate_avpvs_video_dimensions(*args) == want


@pytest.mark.parametrize("args,want", FX["set_pix_fmt"])
def test_set_pix_fmt(args, want):
    src_fmt, codec, encoder, forced, youtube = args
    seg = types.SimpleNamespace(src=types.SimpleNamespace(is_youtube=youtube, stream_info={"pix_fmt": src_fmt}),
                                quality_level=types.SimpleNamespace(video_codec=codec),
                                video_coding=types.SimpleNamespace(encoder=encoder, forced_pix_fmt=forced),
                                target_pix_fmt=None)
    r = _call(chain.set_pix_fmt, seg)
    assert (r if isinstance(r, dict) else seg.target_pix_fmt) == want


@pytest.mark.parametrize("args,want", FX["cpvs_codec"])
def test_cpvs_codec(args, want):
    fmt, raw = args
    pvs = types.SimpleNamespace(segments=[types.SimpleNamespace(target_pix_fmt=fmt)])
    pvs.get_pix_fmt_for_avpvs = types.MethodType(chain.get_pix_fmt_for_avpvs, pvs)
    assert list(chain.get_vcodec_and_pix_fmt_for_cpvs(pvs, rawvideo=raw)) == want


@pytest.mark.parametrize("events,media,dur,bstr", FX["buff_events"])
def test_buff_events(events, media, dur, bstr):
    hrc = ref_stubs.Hrc([tuple(e) for e in events])
    assert chain.hrc_get_buff_events_media_time(hrc) == media
    assert chain.buffer_string(chain.hrc_get_buff_events_media_time(hrc)) == bstr
    assert _call(hrc.get_long_hrc_duration) == dur


@pytest.mark.parametrize("args,want", FX["get_fps"])
def test_get_fps(args, want):
    src_fps, spec = args
    seg = types.SimpleNamespace(quality_level=types.SimpleNamespace(fps=spec),
                                src=types.SimpleNamespace(get_fps=lambda: src_fps))
    r = _call(chain.get_fps, seg)
    assert (r if isinstance(r, dict) else list(r)) == want


@pytest.mark.parametrize("sc,want,venc", FX["encode_segment"])
def test_encode_segment_filter_chain(sc, want, venc):
    seg = scenarios.encode_segment_stub(sc)
    chain_str = chain.encode_segment_filter_chain(seg)
    assert ("-filter:v " + chain_str + " ") in want


@pytest.mark.parametrize("sc,want,venc", FX["encode_segment"])
def test_encode_segment_ffmpeg_backend_identical(sc, want, venc):
    """pixpath.ffmpeg.encode_segment == the reference's string, with the
    reference's own encoder options (what lib/ffmpeg.py hands the drop-in)."""
    pff.set_backend("ffmpeg")
    got = pff.encode_segment(scenarios.encode_segment_stub(sc), overwrite=True,
                             video_encoder_command=lambda seg, **kw: venc)
    assert got == want


@pytest.mark.parametrize("sc,want,venc", FX["encode_segment"])
def test_encode_segment_gpu_backend(sc, want, venc):
    """GPU backend: decode + trim + scale on the MI355X + select/fps on the host
    in `pixpath.cli encseg`, then the reference's encoder options on Y4M."""
    import shlex
    pff.set_backend("gpu")
    try:
        got = pff.encode_segment(scenarios.encode_segment_stub(sc), overwrite=True,
                                 video_encoder_command=lambda seg, **kw: venc)
    finally:
        pff.set_backend("ffmpeg")
    dec, enc = got.split(" | ")
    a = shlex.split(dec)
    assert a[a.index("--width") + 1] == str(sc["ql"][0]) and a[a.index("--pix-fmt") + 1] == sc["pix"]
    assert a[a.index("--in-fps") + 1] == str(sc["src_fps"]) and a[-1] == "-"
    seg = scenarios.encode_segment_stub(sc)
    fps_cmd, fps = chain.get_fps(seg)
    sel = chain.select_expression(float(sc["src_fps"]), fps) if fps_cmd else ""
    assert a[a.index("--select") + 1] == sel
    assert float(a[a.index("--fps") + 1]) == float(fps if fps_cmd else sc["src_fps"])
    assert enc.startswith("ffmpeg -nostdin -y -f yuv4mpegpipe -i - -video_track_timescale 90000 ")
    assert " ".join(venc.split()) in enc and enc.endswith(seg.get_filename())


@pytest.mark.parametrize("i", range(len(FX["builders"])))
def test_builders_ffmpeg_backend(i, tmp_path):
    sc, want, want_list = FX["builders"][i]
    pff.set_backend("ffmpeg")
    root = "/db"
    if sc.get("existing_output"):
        root = str(tmp_path)
    tc, pvs, pps = ref_stubs.build(sc, root, Methods)
    if sc.get("existing_output"):
        for d in ("avpvs", "cpvs"):
            os.makedirs(os.path.join(root, d), exist_ok=True)
        for p in (pvs.get_avpvs_file_path(), pvs.get_avpvs_wo_buffer_file_path(), pvs.get_tmp_wo_audio_path(),
                  pvs.segments[0].get_tmp_path(), pvs.get_cpvs_file_path("pc"),
                  pvs.get_cpvs_file_path(pps[0].processing_type)):
            open(p, "w").close()
    kw = dict(sc.get("kwargs", {}))
    fn = sc["fn"]
    if fn == "create_avpvs_long_concat":
        tc.root = str(tmp_path)
        os.makedirs(os.path.join(str(tmp_path), "avpvs"), exist_ok=True)
        got = pff.create_avpvs_long_concat(pvs, **kw)
        got = got.replace(str(tmp_path), root) if got else got
        lst = open(pvs.get_avpvs_file_list()).read().replace(str(tmp_path), root)
        # segment tmp paths were bound at build time under /db
        assert lst == want_list
    elif fn == "create_avpvs_short":
        got = pff.create_avpvs_short(pvs, **kw)
    elif fn == "create_avpvs_segment":
        got = pff.create_avpvs_segment(pvs.segments[sc.get("seg", 0)], pvs, **kw)
    elif fn == "audio_mux":
        got = pff.audio_mux(pvs, **kw)
    elif fn == "create_cpvs":
        got = pff.create_cpvs(pvs, pps[sc.get("pp", 0)], **kw)
    elif fn == "create_preview":
        got = pff.create_preview(pvs, **kw)
    if got is not None and sc.get("existing_output"):
        got = got.replace(root, "/db")
    assert got == want


def test_bufferer_string_matches_survey_dry_run():
    """SURVEY.md Appendix A a8 (captured from a dry run of p03.run)."""
    pff.set_backend("ffmpeg")
    sc = {"type": "long", "src": [3840, 2160], "segments": [[1280, 720, 2], [1280, 720, 2]], "pps": [["pc", 1920, 1080]],
          "target_pix_fmt": "yuv422p10le", "events": [["quality_level", 4], ["stall", 1.5], ["quality_level", 4]],
          "pvs_id": "P2LXM00_SRC001_HRC001"}
    tc, pvs, _ = ref_stubs.build(sc, "db/P2LXM00", Methods)
    got = pff.bufferer_command(pvs, "/root/reference/util/spinner-128-white.png", force=True)
    assert got == ("bufferer -i db/P2LXM00/avpvs/P2LXM00_SRC001_HRC001_concat_wo_buffer.avi -o "
                   "db/P2LXM00/avpvs/P2LXM00_SRC001_HRC001.avi -b [[4,1.5]] --force-framerate --black-frame -v ffv1 "
                   "-a pcm_s16le -x yuv422p10le -s /root/reference/util/spinner-128-white.png -f")


@pytest.mark.parametrize("row,want", FX["get_difficulty"])
def test_complexity_formula(row, want):
    from pixpath import siti as psiti
    info = {"file_size": row["size"], "video_duration": row["duration"], "video_frame_rate": row["framerate"],
            "video_width": row["width"], "video_height": row["height"]}
    got = psiti.difficulty_from_info("/x/" + row["file"], info)
    assert got == want
    # and the CSV the reference ships was produced by the same formula
    assert abs(got["norm_bitrate"] - row["norm_bitrate"]) <= 3e-15 * row["norm_bitrate"]
    assert abs(got["complexity"] - row["complexity"]) <= 3e-15 * abs(row["complexity"]) + 1e-15


@pytest.mark.parametrize("args,want", FX["classify_complexity"])
def test_classify_complexity(args, want):
    from pixpath import siti as psiti
    c, fr, q = args
    quants = {"low": {0.25: q[0], 0.5: q[1], 0.75: q[2]}, "high": {0.25: q[3], 0.5: q[4], 0.75: q[5]}}
    assert psiti.classify_complexity(c, fr, quants) == want


def test_gpu_backend_strings(tmp_path):
    """GPU backend: one pixpath.cli command per builder, same skip/overwrite rules."""
    pff.set_backend("gpu")
    try:
        sc = FX["builders"][0][0]
        tc, pvs, pps = ref_stubs.build(sc, "/db", Methods)
        s = pff.create_avpvs_short(pvs, overwrite=True)
        assert "-m pixpath.cli avpvs -y --input /db/videoSegments/" in s and "--size 1920x1080" in s
        assert s.endswith("/db/avpvs/P2SXM00_SRC001_HRC001.avi")
        c = pff.create_cpvs(pvs, pps[0], overwrite=True)
        assert "-m pixpath.cli cpvs" in c and "--vcodec rawvideo --pix-fmt uyvy422" in c
        # existing output + no overwrite -> None (lib/ffmpeg.py:964-970)
        tc2, pvs2, _ = ref_stubs.build(sc, str(tmp_path), Methods)
        os.makedirs(os.path.join(str(tmp_path), "avpvs"))
        open(pvs2.get_avpvs_file_path(), "w").close()
        assert pff.create_avpvs_short(pvs2, overwrite=False) is None
    finally:
        pff.set_backend("ffmpeg")


def test_gpu_backend_mobile_tablet_cpvs():
    """create_cpvs mobile/tablet (lib/ffmpeg.py:1202-1231), gpu backend: the
    `scale=DW:DH:flags=bicubic` branch runs `cli avpvs` into yuv420p with the
    reference's own x264 options; the pad branch (leading comma, rejected by
    ffmpeg) keeps the reference's string exactly."""
    seen = set()
    for sc, want, _ in FX["builders"]:
        if sc["fn"] != "create_cpvs" or sc["pps"][0][0] not in ("mobile", "tablet"):
            continue
        tc, pvs, pps = ref_stubs.build(sc, "/db", Methods)
        pff.set_backend("gpu")
        try:
            got = pff.create_cpvs(pvs, pps[sc.get("pp", 0)], **sc.get("kwargs", {}))
        finally:
            pff.set_backend("ffmpeg")
        if "',pad=" in want:
            assert got == want
            seen.add("pad")
        else:
            assert "-m pixpath.cli avpvs" in got and "--pix-fmt yuv420p" in got and "--flags bicubic" in got
            dw, dh = sc["pps"][0][1:3]
            assert "--size %dx%d" % (dw, dh) in got
            vo = want[want.index("-c:v libx264"):want.index("faststart") + len("faststart")]
            assert vo in got  # the reference's x264 options, verbatim
            assert got.split()[-1] == want.split()[-1]
            seen.add("scale")
    assert seen == {"pad", "scale"}
