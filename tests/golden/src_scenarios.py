"""Inputs of the SRC-analysis / complexity fixtures (shared by
gen_src_analysis_fixtures.py, which runs the reference on them, and by the
pixpath tests, which run the mirror on the same inputs).

Canned ffprobe answers (tests/golden/fake_ffprobe.py) for synthetic SRC and
segment files; the files themselves are seeded random bytes of fixed sizes
(the reference hashes them, stats them and probes them; it never decodes).
"""
import json
import os

import numpy as np


def _video(codec="h264", w=3840, h=2160, fmt="yuv420p", rate="60/1", **extra):
    s = {"index": 0, "codec_name": codec, "codec_long_name": "H.264 / AVC / MPEG-4 AVC / MPEG-4 part 10",
         "profile": "High", "codec_type": "video", "codec_tag_string": "avc1", "codec_tag": "0x31637661",
         "width": w, "height": h, "coded_width": w, "coded_height": h, "has_b_frames": 2,
         "sample_aspect_ratio": "1:1", "display_aspect_ratio": "16:9", "pix_fmt": fmt, "level": 51,
         "chroma_location": "left", "refs": 1, "is_avc": "true", "nal_length_size": "4",
         "r_frame_rate": rate, "avg_frame_rate": rate, "time_base": "1/15360", "start_pts": 0,
         "start_time": "0.000000", "bits_per_raw_sample": "8", "disposition": {"default": 1, "dub": 0}}
    s.update(extra)
    return s


def _audio(**extra):
    s = {"index": 1, "codec_name": "aac", "codec_type": "audio", "sample_fmt": "fltp", "sample_rate": "48000",
         "channels": 2, "channel_layout": "stereo", "time_base": "1/48000", "start_pts": 0}
    s.update(extra)
    return s


# analyse_src (util/SRC_analysis.py:120-147): basename -> (file bytes, ffprobe db entry, md5 file?, stale yaml?)
SRC = {
    "SRC001.avi": dict(size=65536, md5=None, yaml=None, probe={
        "streams": [_video(rate="60/1", duration="10.000000", bit_rate="1569904", nb_frames="600",
                           duration_ts=153600),
                    _audio(duration="10.000000", bit_rate="128000")],
        "packets": {"v": [1200 + 37 * i for i in range(24)], "a": [371 + i for i in range(10)]}}),
    "SRC002.mp4": dict(size=40000, md5="0123456789abcdef0123456789abcdef", yaml=None, probe={
        "streams": [_video(w=1920, h=1080, fmt="yuv422p10le", rate="60000/1001", duration="10.010000",
                           bits_per_raw_sample="10", profile="High 4:2:2")],
        "packets": {"v": [5000, 4000, 3000], "a": []}}),
    "SRC003.mkv": dict(size=12345, md5=None, yaml=None, probe={
        "streams": [_video(codec="hevc", w=4096, h=2160, fmt="yuv420p10le", rate="24000/1001",
                           tags={"DURATION": "00:00:08.008000000"}, profile="Main 10")],
        "packets": {"v": [700, 800, 900, 1000], "a": [10, 20]}}),
    "SRC004.avi": dict(size=30000, md5=None,
                       yaml={"get_stream_size": {"v": 111111, "a": 2222}, "md5sum": "-",
                             "get_src_info": {"r_frame_rate": "25"}},
                       probe={"streams": [_video(w=1280, h=720, rate="25/1", duration="6.000000")],
                              "packets": {"v": [1, 2, 3], "a": [4]}}),
}

# get_segment_info (lib/ffmpeg.py:433-563) on a Segment-like {filename, file_path}
SEGMENTS = {
    "seg_full.mp4": dict(size=5000, probe={
        "streams": [_video(w=1920, h=1080, duration="10.000000", bit_rate="4000000"),
                    _audio(duration="10.005000", bit_rate="192000")],
        "packets": {"v": [100] * 10, "a": [50] * 4}}),
    "seg_tags.mkv": dict(size=7000, probe={
        "streams": [_video(w=1280, h=720, rate="30/1", profile="Constrained Baseline",
                           tags={"DURATION": "00:00:10.010000000"}),
                    _audio(nb_frames="470", sample_rate="48000")],
        "packets": {"v": [3000, 2000, 1000, 500], "a": [100, 200]}}),
    "seg_packets.ivf": dict(size=9000, probe={
        "streams": [_video(codec="vp9", w=3840, h=2160, rate="60/1", profile="Profile 0")],
        "packets": {"v": [8000, 1000]},
        "vfi": [{"pts_time": "0.000000", "dts_time": "0.000000", "duration_time": "0.016667", "size": "8000",
                 "flags": "K_"},
                {"pts_time": "0.016667", "dts_time": "0.016667", "duration_time": "0.016667", "size": "1000",
                 "flags": "__"},
                {"pts_time": "0.033333", "size": "900", "flags": "__"}]}),
    "seg_zero.mp4": dict(size=100, probe={"streams": [_video(duration="0.000000", bit_rate="1")], "packets": {}}),
    "seg_novideo.m4a": dict(size=100, probe={"streams": [_audio(duration="1.0", bit_rate="1")], "packets": {}}),
}

# complexity_classification.main(): -i inputs (SRC .avi; one .mp4 is skipped by the
# reference), tmp dir with existing <base>_crf23.avi (size, fps, w, h, duration)
COMPLEXITY_INPUTS = ["SRC101.avi", "SRC102.avi", "SRC103.avi", "SRC104.avi", "SRC105.avi", "SRC106.avi",
                     "SRC107.avi", "SRC108.mp4"]
COMPLEXITY_CRF = {
    "SRC101_crf23.avi": (180000, "60/1", 3840, 2160, "10.000000"),
    "SRC102_crf23.avi": (90000, "60/1", 3840, 2160, "10.000000"),
    "SRC103_crf23.avi": (45000, "30/1", 3840, 2160, "10.000000"),
    "SRC104_crf23.avi": (300000, "60000/1001", 3840, 2160, "10.010000"),
    "SRC105_crf23.avi": (22000, "24/1", 3840, 2160, "8.000000"),
    "SRC106_crf23.avi": (70000, "30/1", 3840, 2160, "10.000000"),
    "SRC107_crf23.avi": (120000, "25/1", 3840, 2160, "10.000000"),
}


def file_bytes(name, size):
    seed = sum(ord(c) * (i + 1) for i, c in enumerate(name))
    return np.random.default_rng(seed).integers(0, 256, size, dtype=np.uint8).tobytes()


def materialise(root):
    """Write every synthetic file and the fake-ffprobe database into `root`;
    returns the database path."""
    db = {}
    for name, sc in SRC.items():
        open(os.path.join(root, name), "wb").write(file_bytes(name, sc["size"]))
        if sc["md5"]:
            open(os.path.join(root, name + ".md5"), "w").write(sc["md5"] + " " + name + "\n")
        if sc["yaml"]:
            import yaml
            with open(os.path.join(root, name + ".yaml"), "w") as f:
                yaml.dump(sc["yaml"], f, default_flow_style=False)
        db[name] = sc["probe"]
    for name, sc in SEGMENTS.items():
        open(os.path.join(root, name), "wb").write(file_bytes(name, sc["size"]))
        db[name] = sc["probe"]
    for name in COMPLEXITY_INPUTS:
        open(os.path.join(root, name), "wb").write(file_bytes(name, 64))
    os.makedirs(os.path.join(root, "complexity"), exist_ok=True)
    for name, (size, rate, w, h, dur) in COMPLEXITY_CRF.items():
        open(os.path.join(root, "complexity", name), "wb").write(file_bytes(name, size))
        db[name] = {"streams": [_video(w=w, h=h, rate=rate, duration=dur, bit_rate=str(size * 8 // 10))],
                    "packets": {"v": [size // 2, size - size // 2]}}
    path = os.path.join(root, "ffprobe_db.json")
    json.dump(db, open(path, "w"))
    return path


def fake_ffprobe_dir(root):
    """A directory holding an executable `ffprobe` that runs fake_ffprobe.py."""
    import stat
    import sys
    d = os.path.join(root, "bin")
    os.makedirs(d, exist_ok=True)
    exe = os.path.join(d, "ffprobe")
    here = os.path.dirname(os.path.abspath(__file__))
    open(exe, "w").write("#!/bin/sh\nexec %s %s \"$@\"\n" % (sys.executable, os.path.join(here, "fake_ffprobe.py")))
    os.chmod(exe, os.stat(exe).st_mode | stat.S_IEXEC | stat.S_IXGRP | stat.S_IXOTH)
    return d
