"""Scenario inputs shared by tests/golden/gen_reference_fixtures.py (which runs
the reference on them) and the host-logic tests (which run pixpath on them)."""
import csv
import os
import types

# calculate_avpvs_video_dimensions(SRC_w, SRC_h, pp_w, pp_h) -- incl. SURVEY a1 cases
DIMS = [
    (3840, 2160, 1920, 1080), (1280, 720, 1920, 1080), (3840, 1600, 1920, 1080), (4096, 2160, 1920, 1080),
    (3840, 2160, 1280, 720), (1920, 800, 1920, 1080), (1920, 1080, 1920, 1080), (1920, 1080, 1280, 800),
    (3840, 2160, 2560, 1440), (4096, 1716, 1920, 1080), (1920, 1080, 3840, 2160), (720, 576, 1920, 1080),
    (3840, 2160, 1080, 1920), (2048, 858, 1280, 720), (3840, 2160, 1024, 768), (3840, 2076, 1280, 800),
    (1080, 1080, 1920, 1080), (1920, 1080, 1920, 1200), (7680, 4320, 3840, 2160), (1000, 1000, 1000, 1000),
]

# Segment.set_pix_fmt inputs: (src pix_fmt, QL codec, encoder, forced_pix_fmt, is_youtube)
SET_PIX_FMT = [
    ("yuv420p", "h264", "libx264", None, False), ("yuv422p", "h264", "libx264", None, False),
    ("yuv444p", "h265", "libx265", None, False), ("yuv420p10le", "h265", "libx265", None, False),
    ("yuv422p10le", "vp9", "libvpx-vp9", None, False), ("yuv444p10le", "av1", "libaom-av1", None, False),
    ("rgb24", "h264", "libx264", None, False), ("gbrp10le", "h264", "libx264", None, False),
    ("yuv422p10le", "h264", "bitmovin", None, False), ("yuv422p10le", "h264", "Bitmovin", None, False),
    ("yuv420p", "h264", "libx264", "yuv444p", False), ("yuv422p10le", "h264", "libx264", None, True),
    ("yuvj420p", "h264", "libx264", None, False), ("yuv410p", "h264", "libx264", None, False),
]

AVPVS_FMTS = ["yuv420p", "yuv422p", "yuv420p10le", "yuv422p10le"]

# Hrc event lists: (event_type, duration)
BUFF_EVENTS = [
    [("quality_level", 8), ("stall", 2.5), ("quality_level", 8), ("stall", 1), ("quality_level", 4)],
    [("freeze", [3, 0.5]), ("quality_level", 10), ("freeze", [1, 0.25])],
    [("quality_level", 4), ("stall", 1.5), ("quality_level", 4)],
    [("stall", 2), ("quality_level", 6), ("quality_level", 6)],
    [("quality_level", 10)],
    [("quality_level", 2), ("stall", 1.5), ("quality_level", 2), ("stall", 1.0), ("quality_level", 2)],
]

# _get_fps(segment): (SRC fps, QL fps spec)
FPS_SPECS = [
    (60, "original"), (60, "auto"), (60, 30), (60, "30"), (30, "24/25/30"), (60, "24/25/30"), (50, "24/25/30"),
    (120, "24/25/30"), (60, "50/60"), (120, "50/60"), (60, "1/2"), (24, "1/2"), (60, "2/5"), (60, 15),
    (50, "30/100"), (25, 15), (24, 15), (30, 24), (60, 20), (24, 8),
]

# encode_segment scenarios: src dims/fps, QL w/h/fps spec
ENCODE_SEGMENT = [
    {"src": [3840, 2160], "src_fps": 60, "ql": [1920, 1080, "original"], "pix": "yuv422p10le"},
    {"src": [3840, 2160], "src_fps": 60, "ql": [1280, 720, 30], "pix": "yuv420p"},
    {"src": [3840, 2160], "src_fps": 60, "ql": [960, 540, "24/25/30"], "pix": "yuv420p"},
    {"src": [3840, 2160], "src_fps": 60, "ql": [640, 360, 15], "pix": "yuv420p"},
    {"src": [3840, 2160], "src_fps": 60, "ql": [1920, 1080, 24], "pix": "yuv420p"},
    {"src": [3840, 2160], "src_fps": 24, "ql": [1920, 1080, 15], "pix": "yuv420p"},
    {"src": [3840, 1600], "src_fps": 50, "ql": [1920, 800, 25], "pix": "yuv422p10le"},
]


def encode_segment_stub(sc):
    tc = types.SimpleNamespace(get_video_segments_path=lambda: "/db/videoSegments",
                               get_logs_path=lambda: "/db/logs", type="short")
    src = types.SimpleNamespace(test_config=tc, file_path="/db/srcVid/SRC001.avi",
                                stream_info={"r_frame_rate": str(sc["src_fps"])},
                                get_fps=lambda: float(sc["src_fps"]))
    ql = types.SimpleNamespace(width=sc["ql"][0], height=sc["ql"][1], fps=sc["ql"][2], video_codec="h264",
                               video_bitrate=8000, video_crf=None, video_qp=None)
    vc = types.SimpleNamespace(passes=1, crf=None, qp=None, encoder="libx264", quality=None, speed=None,
                               scenecut=True, preset="fast", bframes=None, iframe_interval=1, enc_options=None,
                               maxrate_factor=None, bufsize_factor=None, minrate_factor=None)
    seg = types.SimpleNamespace(src=src, quality_level=ql, video_coding=vc, target_pix_fmt=sc["pix"],
                                target_video_bitrate=8000, start_time=0, duration=10, ext="mp4",
                                get_filename=lambda: "DB_SRC001_Q0_VC01_0000_0-10.mp4")
    return seg


def _pp(t, dw, dh, cw=None, ch=None):
    return [t, dw, dh, cw, ch]


PC = _pp("pc", 1920, 1080)
BUILDERS = [
    # --- a2 create_avpvs_short
    {"fn": "create_avpvs_short", "src": [3840, 2160], "segments": [[1280, 720, 10]], "pps": [PC],
     "target_pix_fmt": "yuv420p", "kwargs": {"overwrite": True}},
    {"fn": "create_avpvs_short", "src": [3840, 2160], "src_pix_fmt": "yuv422p10le", "segments": [[1280, 720, 10]],
     "pps": [PC], "target_pix_fmt": "yuv422p10le", "kwargs": {"overwrite": False}},
    {"fn": "create_avpvs_short", "src": [3840, 1600], "segments": [[1280, 534, 10]], "pps": [PC],
     "target_pix_fmt": "yuv420p", "kwargs": {"overwrite": True}},
    {"fn": "create_avpvs_short", "src": [4096, 2160], "segments": [[1920, 1012, 10]], "pps": [PC],
     "target_pix_fmt": "yuv420p10le", "kwargs": {"overwrite": True}},
    {"fn": "create_avpvs_short", "src": [1920, 1080], "segments": [[3840, 2160, 10]], "pps": [PC],
     "target_pix_fmt": "yuv420p", "kwargs": {"overwrite": True}},
    {"fn": "create_avpvs_short", "src": [3840, 2160], "segments": [[1280, 720, 10]], "pps": [PC],
     "target_pix_fmt": "yuv422p10le", "events": [["quality_level", 4], ["stall", 1.5], ["quality_level", 6]],
     "kwargs": {"overwrite": True}},
    {"fn": "create_avpvs_short", "src": [3840, 2160], "src_fps": 50, "segments": [[1280, 720, 10]], "pps": [PC],
     "target_pix_fmt": "yuv422p10le", "kwargs": {"overwrite": True, "scale_avpvs_tosource": True}},
    {"fn": "create_avpvs_short", "src": [3840, 2160], "segments": [[1280, 720, 10]], "pps": [PC],
     "target_pix_fmt": "yuv420p", "kwargs": {"overwrite": True, "force_60_fps": True}},
    {"fn": "create_avpvs_short", "src": [3840, 2160], "segments": [[1280, 720, 10]],
     "pps": [PC, _pp("mobile", 1280, 720)], "target_pix_fmt": "yuv420p",
     "kwargs": {"overwrite": True, "post_proc_id": 1}},
    {"fn": "create_avpvs_short", "src": [3840, 2160], "segments": [[1280, 720, 10]], "pps": [PC],
     "target_pix_fmt": "yuv420p", "kwargs": {"overwrite": False}, "existing_output": True},
    # --- a3 create_avpvs_segment (long tests)
    {"fn": "create_avpvs_segment", "type": "long", "src": [3840, 2160], "src_pix_fmt": "yuv420p10le",
     "segments": [[1280, 720, 4], [1920, 1080, 4]], "pps": [PC], "target_pix_fmt": "yuv420p10le",
     "kwargs": {"overwrite": True}},
    {"fn": "create_avpvs_segment", "type": "long", "src": [3840, 2160], "segments": [[1280, 720, 2], [640, 360, 2]],
     "pps": [PC], "target_pix_fmt": "yuv422p10le", "seg": 1, "kwargs": {"overwrite": False}},
    {"fn": "create_avpvs_segment", "type": "long", "src": [3840, 2160], "src_fps": 30,
     "segments": [[1280, 720, 2]], "pps": [PC], "target_pix_fmt": "yuv420p",
     "kwargs": {"overwrite": True, "scale_avpvs_tosource": True}},
    {"fn": "create_avpvs_segment", "type": "long", "src": [3840, 2160], "segments": [[1280, 720, 2]],
     "pps": [PC], "target_pix_fmt": "yuv420p", "kwargs": {"overwrite": False}, "existing_output": True},
    # --- a4 concat + audio mux
    {"fn": "create_avpvs_long_concat", "type": "long", "src": [3840, 2160],
     "segments": [[1280, 720, 4], [1920, 1080, 4], [640, 360, 4]], "pps": [PC], "target_pix_fmt": "yuv420p",
     "kwargs": {"overwrite": True}},
    {"fn": "create_avpvs_long_concat", "type": "long", "src": [3840, 2160],
     "segments": [[1280, 720, 2.5], [1920, 1080, 2]], "pps": [PC], "target_pix_fmt": "yuv420p",
     "kwargs": {"overwrite": False}},
    {"fn": "audio_mux", "type": "long", "src": [3840, 2160], "segments": [[1280, 720, 4]], "pps": [PC],
     "target_pix_fmt": "yuv420p", "kwargs": {"overwrite": True}},
    {"fn": "audio_mux", "type": "long", "src": [3840, 2160], "segments": [[1280, 720, 4]], "pps": [PC],
     "target_pix_fmt": "yuv420p", "events": [["quality_level", 4], ["stall", 1.5]], "kwargs": {"overwrite": False}},
    # --- a5/a6 create_cpvs
    {"fn": "create_cpvs", "src": [3840, 2160], "segments": [[1280, 720, 10]], "pps": [PC],
     "target_pix_fmt": "yuv420p", "kwargs": {"overwrite": True}},
    {"fn": "create_cpvs", "src": [3840, 2160], "segments": [[1280, 720, 10]], "pps": [PC],
     "target_pix_fmt": "yuv422p10le", "kwargs": {"overwrite": True}},
    {"fn": "create_cpvs", "src": [3840, 2160], "segments": [[1280, 720, 10]], "pps": [PC],
     "target_pix_fmt": "yuv420p10le", "kwargs": {"overwrite": False}},
    {"fn": "create_cpvs", "src": [3840, 2160], "segments": [[1280, 720, 10]], "pps": [PC],
     "target_pix_fmt": "yuv422p", "kwargs": {"overwrite": True, "rawvideo": True}},
    {"fn": "create_cpvs", "src": [3840, 1600], "segments": [[1280, 534, 10]], "pps": [PC],
     "target_pix_fmt": "yuv420p", "kwargs": {"overwrite": True}},
    {"fn": "create_cpvs", "src": [4096, 2160], "segments": [[1920, 1012, 10]], "pps": [PC],
     "target_pix_fmt": "yuv422p10le", "kwargs": {"overwrite": True}},
    {"fn": "create_cpvs", "type": "long", "src": [3840, 2160], "segments": [[1280, 720, 4], [1920, 1080, 4]],
     "pps": [PC], "target_pix_fmt": "yuv420p", "events": [["quality_level", 4], ["stall", 1.5], ["quality_level", 4]],
     "kwargs": {"overwrite": True}},
    {"fn": "create_cpvs", "src": [3840, 2160], "segments": [[1280, 720, 10]], "pps": [_pp("tablet", 1280, 800, 1280, 720)],
     "target_pix_fmt": "yuv420p", "kwargs": {"overwrite": True}},
    {"fn": "create_cpvs", "src": [3840, 2160], "segments": [[1280, 720, 10]], "pps": [_pp("mobile", 1280, 720)],
     "target_pix_fmt": "yuv420p", "kwargs": {"overwrite": True, "nonraw_crf": 20, "mobile_preset": "slow"}},
    {"fn": "create_cpvs", "type": "long", "src": [3840, 2160], "segments": [[1280, 720, 4]],
     "pps": [_pp("mobile", 1280, 720)], "target_pix_fmt": "yuv420p", "kwargs": {"overwrite": True}},
    {"fn": "create_cpvs", "src": [3840, 1600], "segments": [[1280, 534, 10]], "pps": [_pp("hd-pc-home", 1920, 1080)],
     "target_pix_fmt": "yuv420p", "kwargs": {"overwrite": True}},
    {"fn": "create_cpvs", "src": [3840, 2160], "segments": [[1280, 720, 10]], "pps": [PC],
     "target_pix_fmt": "yuv420p", "kwargs": {"overwrite": False}, "existing_output": True},
    {"fn": "create_preview", "src": [3840, 2160], "segments": [[1280, 720, 10]], "pps": [PC],
     "target_pix_fmt": "yuv420p", "kwargs": {"overwrite": True}},
]

# classify_complexity(complexity, framerate, quantiles low(25,50,75) + high(25,50,75))
CLASSIFY = [
    (3.0, 24.0, [2.0, 4.0, 6.0, 1.0, 2.0, 3.0]), (5.0, 24.0, [2.0, 4.0, 6.0, 1.0, 2.0, 3.0]),
    (7.0, 30.0, [2.0, 4.0, 6.0, 1.0, 2.0, 3.0]), (1.0, 30.0, [2.0, 4.0, 6.0, 1.0, 2.0, 3.0]),
    (2.5, 60.0, [2.0, 4.0, 6.0, 1.0, 2.0, 3.0]), (4.0, 60.0, [2.0, 4.0, 6.0, 1.0, 2.0, 3.0]),
    (2.0, 24.0, [2.0, 4.0, 6.0, 1.0, 2.0, 3.0]), (4.0, 24.0, [2.0, 4.0, 6.0, 1.0, 2.0, 3.0]),
]


def complexity_rows(golden_dir):
    rows = []
    for name in ("complexity_classification.csv", "complexity_classification_validation.csv"):
        with open(os.path.join(golden_dir, name)) as f:
            for r in csv.DictReader(f):
                rows.append({"file": r["file"], "size": int(r["size"]), "duration": float(r["duration"]),
                             "framerate": float(r["framerate"]), "width": int(r["width"]),
                             "height": int(r["height"]), "norm_bitrate": float(r["norm_bitrate"]),
                             "complexity": float(r["complexity"]), "complexity_class": int(r["complexity_class"])})
    return rows
