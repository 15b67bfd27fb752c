#!/usr/bin/env python3
"""Generate tests/golden/reference_fixtures.json by running the REFERENCE's own
Python (pnats2avhd/processing-chain, read-only at $REFERENCE, default
/root/reference) on the scenarios of tests/golden/scenarios.py.

Only run in the build container (the reference does not travel to the GPU box);
the JSON it writes is data: scenario inputs and the reference's outputs
(command strings, AVPVS dims, pixel-format decisions, stall schedules,
complexity numbers).  Nothing of the reference's source is copied.

Reference functions exercised (file:line):
  lib/ffmpeg.py:33    calculate_avpvs_video_dimensions
  lib/ffmpeg.py:321   _get_fps                    (fps / select decision, a14)
  lib/ffmpeg.py:772   encode_segment              (p01 scale/select/fps chain, a7)
  lib/ffmpeg.py:940   create_avpvs_short          (a2)
  lib/ffmpeg.py:1003  create_avpvs_segment        (a3)
  lib/ffmpeg.py:1058  create_avpvs_long_concat    (a4)
  lib/ffmpeg.py:1149  create_cpvs                 (a5, a6)
  lib/ffmpeg.py:1250  create_preview
  lib/ffmpeg.py:1262  audio_mux                   (a4)
  lib/test_config.py:172  Pvs.get_pix_fmt_for_avpvs          (a9)
  lib/test_config.py:188  Pvs.get_vcodec_and_pix_fmt_for_cpvs (a9)
  lib/test_config.py:312  Hrc.get_buff_events_media_time     (a10)
  lib/test_config.py:447  Segment.set_pix_fmt                (a9)
  util/complexity_classification.py:50,72  get_difficulty, classify_complexity (a12)
"""
import json
import os
import sys
import tempfile
import types

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))  # tests/
REFERENCE = os.environ.get("REFERENCE", "/root/reference")

import ref_stubs  # noqa: E402
import scenarios  # noqa: E402


def call(fn, *a, **k):
    """Run a reference function; encode its failure conventions as data."""
    try:
        return fn(*a, **k)
    except SystemExit as e:  # logger.error + sys.exit(1)
        return {"sys_exit": e.code}
    except Exception as e:  # a crash of the reference itself
        return {"error": type(e).__name__}


def main():
    sys.path.insert(0, REFERENCE)
    sys.path.insert(0, os.path.join(REFERENCE, "util"))
    import lib.ffmpeg as rff
    import lib.test_config as rtc
    import complexity_classification as rcc

    class RefMethods:
        get_pix_fmt_for_avpvs = rtc.Pvs.get_pix_fmt_for_avpvs
        get_vcodec_and_pix_fmt_for_cpvs = rtc.Pvs.get_vcodec_and_pix_fmt_for_cpvs
        get_buff_events_media_time = rtc.Pvs.get_buff_events_media_time
        hrc_get_buff_events_media_time = rtc.Hrc.get_buff_events_media_time

    out = {"generator": "tests/golden/gen_reference_fixtures.py", "reference": "pnats2avhd/processing-chain 1.0.0"}

    out["avpvs_dims"] = [[list(a), rff.calculate_avpvs_video_dimensions(*a)] for a in scenarios.DIMS]

    # Segment.set_pix_fmt on duck-typed segments
    pf = []
    for src_fmt, codec, encoder, forced, youtube in scenarios.SET_PIX_FMT:
        seg = types.SimpleNamespace(
            src=types.SimpleNamespace(is_youtube=youtube, stream_info={"pix_fmt": src_fmt}),
            quality_level=types.SimpleNamespace(video_codec=codec),
            video_coding=types.SimpleNamespace(encoder=encoder, forced_pix_fmt=forced),
            target_pix_fmt=None)
        seg.src.uses_10_bit = types.MethodType(rtc.Src.uses_10_bit, seg.src)
        try:
            rtc.Segment.set_pix_fmt(seg)
            res = seg.target_pix_fmt
        except SystemExit as e:  # the reference's error convention: logger.error + sys.exit(1)
            res = {"sys_exit": e.code}
        pf.append([[src_fmt, codec, encoder, forced, youtube], res])
    out["set_pix_fmt"] = pf

    cp = []
    for fmt in scenarios.AVPVS_FMTS:
        for raw in (False, True):
            pvs = types.SimpleNamespace(segments=[types.SimpleNamespace(target_pix_fmt=fmt)])
            pvs.get_pix_fmt_for_avpvs = types.MethodType(rtc.Pvs.get_pix_fmt_for_avpvs, pvs)
            cp.append([[fmt, raw], list(rtc.Pvs.get_vcodec_and_pix_fmt_for_cpvs(pvs, rawvideo=raw))])
    out["cpvs_codec"] = cp

    be = []
    for events in scenarios.BUFF_EVENTS:
        hrc = ref_stubs.Hrc(events)
        be.append([events, call(rtc.Hrc.get_buff_events_media_time, hrc), call(rtc.Hrc.get_long_hrc_duration, hrc),
                   str(rtc.Hrc.get_buff_events_media_time(hrc)).replace(" ", "")])
    out["buff_events"] = be

    fps = []
    for src_fps, spec in scenarios.FPS_SPECS:
        seg = types.SimpleNamespace(quality_level=types.SimpleNamespace(fps=spec),
                                    src=types.SimpleNamespace(get_fps=lambda f=src_fps: f))
        try:
            res = list(rff._get_fps(seg))
        except SystemExit as e:
            res = {"sys_exit": e.code}
        fps.append([[src_fps, spec], res])
    out["get_fps"] = fps

    # encode_segment (one-pass libx264) -> the -filter:v chain of a7
    enc = []
    for sc in scenarios.ENCODE_SEGMENT:
        try:
            res = rff.encode_segment(scenarios.encode_segment_stub(sc), overwrite=True)
        except SystemExit as e:
            res = {"sys_exit": e.code}
        # the encoder options (not pixel work): what the drop-in receives from
        # the reference's _get_video_encoder_command
        venc = call(rff._get_video_encoder_command, scenarios.encode_segment_stub(sc))
        enc.append([sc, res, venc])
    out["encode_segment"] = enc

    # command builders
    builders = []
    for sc in scenarios.BUILDERS:
        root = sc.get("root", "/db")
        tmp = None
        if sc.get("existing_output"):
            tmp = tempfile.mkdtemp()
            root = tmp
        tc, pvs, pps = ref_stubs.build(sc, root, RefMethods)
        if tmp:
            for d in ("avpvs", "cpvs"):
                os.makedirs(os.path.join(tmp, d), exist_ok=True)
            for p in (pvs.get_avpvs_file_path(), pvs.get_avpvs_wo_buffer_file_path(),
                      pvs.get_tmp_wo_audio_path(), pvs.segments[0].get_tmp_path(),
                      pvs.get_cpvs_file_path("pc"), pvs.get_cpvs_file_path(pps[0].processing_type)):
                open(p, "w").close()
        fn = sc["fn"]
        kw = dict(sc.get("kwargs", {}))
        if fn == "create_avpvs_short":
            r = rff.create_avpvs_short(pvs, **kw)
        elif fn == "create_avpvs_segment":
            r = rff.create_avpvs_segment(pvs.segments[sc.get("seg", 0)], pvs, **kw)
        elif fn == "create_avpvs_long_concat":
            # the filelist side effect (lib/ffmpeg.py:1086-1092) is written to a temp dir
            with tempfile.TemporaryDirectory() as d:
                os.makedirs(os.path.join(d, "avpvs"))
                real = tc.get_avpvs_path
                tc.get_avpvs_path = lambda: os.path.join(d, "avpvs")
                lst = pvs.get_avpvs_file_list()
                r = rff.create_avpvs_long_concat(pvs, **kw)
                filelist = open(lst).read() if os.path.exists(lst) else None
                tc.get_avpvs_path = real
                if r is not None:
                    r = r.replace(d, root)
                if filelist is not None:
                    filelist = filelist.replace(d, root)
            builders.append([sc, r, filelist])
            continue
        elif fn == "audio_mux":
            r = rff.audio_mux(pvs, **kw)
        elif fn == "create_cpvs":
            r = rff.create_cpvs(pvs, pps[sc.get("pp", 0)], **kw)
        elif fn == "create_preview":
            r = rff.create_preview(pvs, **kw)
        else:
            raise ValueError(fn)
        if tmp and r is not None:
            r = r.replace(tmp, "/db")
        builders.append([sc, r, None])
    out["builders"] = builders

    # complexity KAT: get_difficulty with the reference's formula, classify_complexity
    kat = []
    for row in scenarios.complexity_rows(HERE):
        info = {"file_size": row["size"], "video_duration": row["duration"], "video_frame_rate": row["framerate"],
                "video_width": row["width"], "video_height": row["height"]}
        rcc.get_segment_info = lambda seg, info=info: info
        kat.append([row, rcc.get_difficulty("/x/" + row["file"])])
    out["get_difficulty"] = kat
    cls = []
    for c, fr, q in scenarios.CLASSIFY:
        quants = {"low": {0.25: q[0], 0.5: q[1], 0.75: q[2]}, "high": {0.25: q[3], 0.5: q[4], 0.75: q[5]}}
        cls.append([[c, fr, q], rcc.classify_complexity(c, fr, quants)])
    out["classify_complexity"] = cls

    path = os.path.join(HERE, "reference_fixtures.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", path, "builders:", len(builders))


if __name__ == "__main__":
    main()
