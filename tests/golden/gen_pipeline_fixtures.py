#!/usr/bin/env python3
"""Generate tests/golden/pipeline_fixtures.json: the REFERENCE's own p03 and
p04 (`--dry-run`) with the reference-side binding of INTEGRATION.md applied,
on a synthetic short and long database -- every command each builder call
returns, in call order, for the ffmpeg backend (the reference unchanged) and
the gpu backend (the binding in effect).

What is applied, read from INTEGRATION.md at generation time:
  section 2: the python block appended to lib/ffmpeg.py -- exec'd in the
             namespace of the imported reference module lib.ffmpeg;
  section 3: the two lines added after p03's inline bufferer string
             (p03_generateAvPvs.py:242-243) -- inserted into the text of
             p03_generateAvPvs.py, compiled and run in memory.
Nothing is written into /root/reference; only the JSON (data: command
strings, with the temp root shown as /db) is committed.

The databases follow SURVEY.md section 4's fake-backend technique: a fake
`ffprobe` on PATH (tests/golden/fake_ffprobe.py) answers for the synthetic
SRC files, the test-config YAML is named like the DB folder (P2SXM00,
P2LXM00; lib/test_config.py:1012, :1081).

Reference entry points exercised (file:line):
  p03_generateAvPvs.py:62   run (short: create_avpvs_short; long:
                            create_avpvs_segment, create_avpvs_long_concat,
                            audio_mux, then the bufferer step :215-254)
  p04_generateCpvs.py:31    run (create_cpvs, create_preview with -e)
  lib/test_config.py:1025   TestConfig (the YAML below)
"""
import json
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REFERENCE = os.environ.get("REFERENCE", "/root/reference")
PKG = os.path.join(REPO, "processing-chain_amd")
INTEGRATION = os.path.join(REPO, "INTEGRATION.md")

BUILDERS = ("create_avpvs_short", "create_avpvs_segment", "create_avpvs_long_concat", "audio_mux", "create_cpvs",
            "create_preview", "bufferer_command")

P03_ANCHOR = "' -v ffv1 -a pcm_s16le -x {pix_fmt} {stalling_type_options} {overwrite_spec}'.format(**locals())\n"


def _video(w, h, fmt, rate="60/1", dur="10.000000"):
    return {"index": 0, "codec_name": "h264", "profile": "High", "codec_type": "video", "width": w, "height": h,
            "coded_width": w, "coded_height": h, "pix_fmt": fmt, "r_frame_rate": rate, "avg_frame_rate": rate,
            "time_base": "1/15360", "duration": dur, "bit_rate": "20000000", "nb_frames": "600"}


def _audio(dur="10.000000"):
    return {"index": 1, "codec_name": "pcm_s16le", "codec_type": "audio", "sample_rate": "48000", "channels": 2,
            "duration": dur, "bit_rate": "1536000"}


# SRC files: name -> ffprobe streams
SRCS = {
    "SRC001.avi": [_video(3840, 2160, "yuv420p"), _audio()],
    "SRC002.avi": [_video(1920, 1080, "yuv422p10le"), _audio()],
    "SRC003.avi": [_video(3840, 2160, "yuv420p10le", dur="12.000000"), _audio("12.000000")],
}

QLS = {"Q0": {"index": 0, "videoCodec": "h264", "videoBitrate": 8000, "width": 1920, "height": 1080, "fps": 60},
       "Q1": {"index": 1, "videoCodec": "h264", "videoBitrate": 2000, "width": 1280, "height": 720, "fps": 60},
       "Q2": {"index": 2, "videoCodec": "h264", "videoBitrate": 1000, "width": 960, "height": 540, "fps": 30}}

SHORT = {
    "databaseId": "P2SXM00", "syntaxVersion": 6, "type": "short",
    "qualityLevelList": QLS,
    "codingList": {"VC01": {"type": "video", "encoder": "libx264", "passes": 1, "iFrameInterval": 1}},
    "srcList": {"SRC001": "SRC001.avi", "SRC002": "SRC002.avi"},
    "hrcList": {"HRC001": {"videoCodingId": "VC01", "eventList": [["Q1", 10]]},
                "HRC002": {"videoCodingId": "VC01", "eventList": [["Q2", 10], ["stall", 1.5]]},
                "HRC003": {"videoCodingId": "VC01", "eventList": [["Q1", 10], ["freeze", [3, 0.5]],
                                                                   ["freeze", [1, 0.25]]]}},
    "pvsList": ["P2SXM00_SRC001_HRC001", "P2SXM00_SRC001_HRC002", "P2SXM00_SRC002_HRC003"],
    "postProcessingList": [{"type": "pc", "displayWidth": 1920, "displayHeight": 1080, "codingWidth": 1920,
                            "codingHeight": 1080}],
}

# config-4 shape: 2-s segments, stalls [[2, 1.5], [4, 1.0]] in media time
LONG = {
    "databaseId": "P2LXM00", "syntaxVersion": 6, "type": "long", "segmentDuration": 2,
    "qualityLevelList": {k: dict(v, audioCodec="aac", audioBitrate=128) for k, v in QLS.items()},
    "codingList": {"VC01": {"type": "video", "encoder": "libx264", "passes": 1, "iFrameInterval": 1},
                   "AC01": {"type": "audio", "encoder": "aac"}},
    "srcList": {"SRC003": "SRC003.avi"},
    "hrcList": {"HRC001": {"videoCodingId": "VC01", "audioCodingId": "AC01",
                           "eventList": [["Q1", 2], ["stall", 1.5], ["Q0", 2], ["stall", 1.0], ["Q1", 2]]}},
    "pvsList": ["P2LXM00_SRC003_HRC001"],
    "postProcessingList": [{"type": "pc", "displayWidth": 1920, "displayHeight": 1080, "codingWidth": 1920,
                            "codingHeight": 1080}],
}


def integration_blocks():
    """(section-2 python block, section-3 python block) of INTEGRATION.md."""
    text = open(INTEGRATION).read()

    def block(heading):
        i = text.index(heading)
        j = text.index("```python\n", i) + len("```python\n")
        return text[j:text.index("```", j)]
    return block("## 2. Reference-side change (lib/ffmpeg.py)"), block("## 3. Reference-side change")


def materialise(root):
    import yaml
    srcdb = {}
    for db in (SHORT, LONG):
        d = os.path.join(root, db["databaseId"])
        os.makedirs(os.path.join(d, "srcVid"))
        with open(os.path.join(d, db["databaseId"] + ".yaml"), "w") as f:
            yaml.safe_dump(db, f, default_flow_style=False)
        for name in db["srcList"].values():
            with open(os.path.join(d, "srcVid", name), "wb") as f:
                f.write(b"\0" * 4096)
            srcdb[name] = {"streams": SRCS[name], "packets": {"v": [1000] * 4, "a": [100] * 4}}
    with open(os.path.join(root, "ffprobe_db.json"), "w") as f:
        json.dump(srcdb, f)
    bind = os.path.join(root, "bin")
    os.makedirs(bind)
    with open(os.path.join(bind, "ffprobe"), "w") as f:
        f.write("#!/bin/sh\nexec %s %s \"$@\"\n" % (sys.executable, os.path.join(HERE, "fake_ffprobe.py")))
    os.chmod(os.path.join(bind, "ffprobe"), 0o755)
    return bind


def inner(root, db_id, backend):
    """In a child process: run p03 then p04 dry on one database, one backend."""
    import types
    sys.path.insert(0, REFERENCE)
    os.chdir(root)
    if backend == "gpu":
        os.environ["PIXPATH_BACKEND"] = "gpu"
        os.environ["PIXPATH_HOME"] = PKG
        os.environ["PIXPATH_FFV1"] = "gpu"
        os.environ["PIXPATH_FFV1_SLICES"] = "8x8"
    else:
        os.environ.pop("PIXPATH_BACKEND", None)
    import lib.cmd_utils as cmd_utils  # noqa: F401
    import lib.ffmpeg as rff
    import lib.parse_args as parse_args
    import lib.test_config as cfg
    sec2, sec3 = integration_blocks()
    exec(compile(sec2, INTEGRATION + ":section2", "exec"), rff.__dict__)
    calls = []

    def wrap(name, fn):
        def rec(*a, **k):
            r = fn(*a, **k)
            calls.append([name, r])
            return r
        return rec
    for name in BUILDERS:
        if hasattr(rff, name):
            setattr(rff, name, wrap(name, getattr(rff, name)))
    scheduled = []  # what the scripts hand to their ParallelRunners (lib/cmd_utils.py:73-79)
    add_cmd = cmd_utils.ParallelRunner.add_cmd

    def rec_add(self, cmd, name=""):
        if cmd:
            scheduled.append([name, cmd])
        return add_cmd(self, cmd, name)
    cmd_utils.ParallelRunner.add_cmd = rec_add
    p03_path = os.path.join(REFERENCE, "p03_generateAvPvs.py")
    src = open(p03_path).read()
    assert src.count(P03_ANCHOR) == 1, "p03 anchor not found"
    src = src.replace(P03_ANCHOR, P03_ANCHOR + sec3)
    p03 = types.ModuleType("p03_generateAvPvs")
    p03.__file__ = p03_path
    exec(compile(src, p03_path, "exec"), p03.__dict__)
    import p04_generateCpvs as p04
    yml = os.path.join(root, db_id, db_id + ".yaml")
    out = {}
    for name, mod, extra in (("p03", p03, []), ("p04", p04, ["-e"])):
        sys.argv = [name, "-c", yml, "-n"] + extra
        ns = parse_args.parse_args(name, int(name[-1]))
        del calls[:]
        del scheduled[:]
        try:
            mod.run(ns, cfg.TestConfig(yml))
        except SystemExit as e:
            assert not e.code, "%s exited %r" % (name, e.code)
        out[name] = [[n, r] for n, r in calls]
        out[name + "_scheduled"] = sorted(scheduled)
    json.dump(out, open(os.path.join(root, "result.json"), "w"))


def normalise(obj, root):
    if isinstance(obj, str):
        s = obj.replace(root, "/db").replace(PKG, "$PIXPATH_HOME").replace(REFERENCE, "$REFERENCE")
        return re.sub(r"'\$PIXPATH_HOME'", "$PIXPATH_HOME", s)
    if isinstance(obj, list):
        return [normalise(x, root) for x in obj]
    if isinstance(obj, dict):
        return {k: normalise(v, root) for k, v in obj.items()}
    return obj


def main():
    sec2, sec3 = integration_blocks()
    res = {"generator": "tests/golden/gen_pipeline_fixtures.py", "reference": "pnats2avhd/processing-chain 1.0.0",
           "integration_section2": sec2, "integration_section3": sec3, "runs": {}}
    with tempfile.TemporaryDirectory() as root:
        root = os.path.realpath(root)
        bind = materialise(root)
        env = dict(os.environ, FAKE_FFPROBE_DB=os.path.join(root, "ffprobe_db.json"),
                   PATH=bind + os.pathsep + os.environ["PATH"])
        for db in (SHORT, LONG):
            for backend in ("ffmpeg", "gpu"):
                p = subprocess.run([sys.executable, os.path.abspath(__file__), "--inner", root, db["databaseId"],
                                    backend], env=env, capture_output=True, text=True)
                if p.returncode:
                    sys.stderr.write(p.stdout[-4000:] + p.stderr[-4000:])
                    raise SystemExit("reference run failed: %s %s" % (db["databaseId"], backend))
                r = json.load(open(os.path.join(root, "result.json")))
                res["runs"]["%s/%s" % (db["databaseId"], backend)] = normalise(r, root)
    path = os.path.join(HERE, "pipeline_fixtures.json")
    json.dump(res, open(path, "w"), indent=1, sort_keys=True)
    print("wrote", path, {k: {s: len(v) for s, v in r.items()} for k, r in res["runs"].items()})


if __name__ == "__main__":
    if len(sys.argv) > 4 and sys.argv[1] == "--inner":
        inner(sys.argv[2], sys.argv[3], sys.argv[4])
    else:
        main()
