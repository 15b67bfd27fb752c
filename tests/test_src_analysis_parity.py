"""SRC-analysis / complexity boundary vs the reference's own outputs (CPU).

tests/golden/src_analysis_fixtures.json holds what the reference produced
(tests/golden/gen_src_analysis_fixtures.py: util/SRC_analysis.analyse_src,
lib/ffmpeg.get_segment_info, util/complexity_classification.main) on the
synthetic files of tests/golden/src_scenarios.py with tests/golden/fake_ffprobe.py
as `ffprobe`.  pixpath runs on the same files with the same fake ffprobe and
must reproduce the reference byte for byte; the SI/TI additions are the only
difference (an extra `siti` YAML key, extra `si`, `ti`, `siti_bitdepth`,
`siti_scale` CSV columns)."""
import contextlib
import io
import json
import os
import sys

import numpy as np
import pytest
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import src_scenarios as sc  # noqa: E402

FX = json.load(open(os.path.join(HERE, "golden", "src_analysis_fixtures.json")))


@pytest.fixture()
def fake_root(tmp_path, monkeypatch):
    db = sc.materialise(str(tmp_path))
    monkeypatch.setenv("FAKE_FFPROBE_DB", db)
    monkeypatch.setenv("PATH", sc.fake_ffprobe_dir(str(tmp_path)) + os.pathsep + os.environ["PATH"])
    monkeypatch.chdir(tmp_path)
    return str(tmp_path)


def _strip_siti(text):
    """YAML text without the top-level `siti:` block."""
    out, skip = [], False
    for line in text.splitlines(keepends=True):
        if line.startswith("siti:"):
            skip = True
            continue
        if skip and line.startswith(" "):
            continue
        skip = False
        out.append(line)
    return "".join(out)


@pytest.mark.parametrize("name", sorted(sc.SRC))
def test_analyse_src_yaml_identical(fake_root, name):
    from pixpath import siti
    ref = FX["analyse_src"][name]
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        yp = siti.analyse_src(os.path.join(fake_root, name), ref["ordernum"], with_siti=False)
    assert os.path.relpath(yp, fake_root) == ref["yaml_path_suffix"]
    assert open(yp).read() == ref["yaml"]
    assert buf.getvalue() == ref["stdout"]


@pytest.mark.parametrize("name", sorted(sc.SRC))
def test_analyse_src_with_siti_adds_only_the_siti_key(fake_root, name):
    from pixpath import siti
    ref = FX["analyse_src"][name]
    si = np.array([10.5, 11.25, 9.0])
    ti = np.array([np.nan, 3.5, 4.0])
    with contextlib.redirect_stdout(io.StringIO()):
        yp = siti.analyse_src(os.path.join(fake_root, name), ref["ordernum"], siti=(si, ti))
    text = open(yp).read()
    assert _strip_siti(text) == ref["yaml"]
    d = yaml.safe_load(text)
    assert d["siti"]["si"] == 11.25 and d["siti"]["ti"] == 4.0
    assert d["siti"]["ti_frames"][0] is None and d["siti"]["si_frames"] == [10.5, 11.25, 9.0]
    with contextlib.redirect_stdout(io.StringIO()):
        yp = siti.analyse_src(os.path.join(fake_root, name), ref["ordernum"], siti=(si, ti), bitdepth=10)
    d = yaml.safe_load(open(yp))
    assert d["siti"]["bitdepth"] == 10 and d["siti"]["scale"] == 1.0 and d["siti"]["normalized"] is False


def test_r_frame_rate_truncates_like_the_reference(fake_root):
    from pixpath import probe
    assert probe.get_src_info(os.path.join(fake_root, "SRC002.mp4"))["r_frame_rate"] == "59"
    assert probe.get_src_info(os.path.join(fake_root, "SRC003.mkv"))["r_frame_rate"] == "23"
    assert probe.get_src_info(os.path.join(fake_root, "SRC001.avi"))["r_frame_rate"] == "60"


def test_stream_size_prefers_existing_yaml(fake_root):
    from pixpath import probe
    p = os.path.join(fake_root, "SRC004.avi")
    assert probe.get_stream_size(p) == 111111 and probe.get_stream_size(p, "audio") == 2222
    assert probe.get_stream_size(os.path.join(fake_root, "SRC001.avi")) == sum(sc.SRC["SRC001.avi"]["probe"]["packets"]["v"])


@pytest.mark.parametrize("name", sorted(sc.SEGMENTS))
def test_get_segment_info_identical(fake_root, name):
    from pixpath import probe
    ref = FX["get_segment_info"][name]
    try:
        got = {"ok": [[k, v] for k, v in probe.get_segment_info(os.path.join(fake_root, name)).items()]}
    except SystemExit as e:
        got = {"sys_exit": e.code}
    assert got == ref


def test_complexity_csv_identical_plus_siti_columns(fake_root):
    """complexity main() mirror: the reference's CSV byte for byte, si/ti appended."""
    import pandas as pd
    from pixpath import siti
    # two SRCs already carry analyse_src YAMLs with SI/TI, the rest have none
    # (SRC104's entry carries its bit depth: 10-bit raw code values)
    for name, e in (("SRC101.avi", {"si": 61.5, "ti": 20.25}),
                    ("SRC104.avi", {"si": 40.0, "ti": 9.5, "bitdepth": 10, "scale": 1.0})):
        with open(os.path.join(fake_root, name + ".yaml"), "w") as f:
            yaml.dump({"md5sum": "-", "siti": e}, f)
    argv = ["-i"] + [os.path.join(fake_root, f) for f in sc.COMPLEXITY_INPUTS] + \
        ["-t", os.path.join(fake_root, "complexity"), "-o", "complexity.csv"]
    csv = siti.complexity_main(argv)
    got = pd.read_csv(csv, float_precision="round_trip")
    extra = ["si", "ti", "siti_bitdepth", "siti_scale"]
    assert list(got.columns[-4:]) == extra
    ref_text = FX["complexity_csv"]
    assert got.drop(columns=extra).to_csv(index=False) == ref_text
    # the exact text: every line is the reference's line plus ",si,ti"
    lines = open(csv).read().splitlines()
    ref_lines = ref_text.splitlines()
    assert lines[0] == ref_lines[0] + ",si,ti,siti_bitdepth,siti_scale"
    for a, b in zip(lines[1:], ref_lines[1:]):
        assert a.startswith(b + ",")
    row = got.set_index("file")
    assert row.loc["SRC101_crf23.avi", "si"] == 61.5 and row.loc["SRC104_crf23.avi", "ti"] == 9.5
    assert np.isnan(row.loc["SRC102_crf23.avi", "si"])
    assert row.loc["SRC104_crf23.avi", "siti_bitdepth"] == 10 and row.loc["SRC104_crf23.avi", "siti_scale"] == 1.0
    assert np.isnan(row.loc["SRC101_crf23.avi", "siti_bitdepth"])
    # the 8-bit scale: SRC104's 10-bit raw values divided by 4, recorded as such
    csv8 = siti.complexity_main(argv + ["--siti-scale", "8bit", "-o", "c8.csv"])
    r8 = pd.read_csv(csv8, float_precision="round_trip").set_index("file")
    assert r8.loc["SRC104_crf23.avi", "si"] == 10.0 and r8.loc["SRC104_crf23.avi", "ti"] == 2.375
    assert r8.loc["SRC104_crf23.avi", "siti_scale"] == 0.25
    assert r8.loc["SRC101_crf23.avi", "si"] == 61.5  # depth unknown: left as written
    csv2 = siti.complexity_main(argv + ["--siti", "none", "-o", "plain.csv"])
    assert open(csv2).read() == ref_text


def test_complexity_dry_run_lists_encodes(fake_root, caplog):
    from pixpath import siti
    with pytest.raises(SystemExit) as e:
        siti.complexity_main(["-i", os.path.join(fake_root, "SRC101.avi"), "-t", os.path.join(fake_root, "fresh"),
                              "-n"])
    assert e.value.code == 0


def test_complexity_tmp_dir_default_is_next_to_the_script(tmp_path):
    """--tmp-dir defaults to complexityAnalysis beside the calling script, as
    the reference's (util/complexity_classification.py:100-105)."""
    import os
    from pixpath import siti
    a = siti.complexity_parse_args(["-i", "x.avi"], script_dir="/opt/pc/util")
    assert a.tmp_dir == os.path.join("/opt/pc/util", "complexityAnalysis")
    b = siti.complexity_parse_args(["-i", "x.avi", "-t", str(tmp_path)])
    assert b.tmp_dir == str(tmp_path)
