"""p02 frame-size scanners against the reference.

* pixpath.framesize.get_framesize_h264/h265/vp9 (native scanner in
  libpixpath, csrc/scan.cpp) return, print and clean up exactly what the
  reference's lib/get_framesize.py did on the same files -- sizes, ValueError
  crashes, "Frame misdeteciton!" lines, the empty-file early return that leaves
  the temp file behind (tests/golden/framesize_fixtures.json, made by
  tests/golden/gen_framesize_fixtures.py from the reference itself);
* delete_packets leaves the same packet list (or raises the same error);
* the oracle restatement (oracle/framesize_ref.py) is pinned by the same
  fixtures, then the native scanner is fuzzed against it on random streams;
* the builders of the synthetic streams have not drifted (SHA-256).
Host-only: no GPU.
"""
import base64
import contextlib
import copy
import io
import json
import os

import numpy as np
import pytest

import framesize_ref as ref
import framesize_streams as fs
from pixpath import framesize

FX = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "framesize_fixtures.json")))
EXT = {"h264": "h264", "h265": "h265", "vp9": "ivf"}


def run_mirror(tmp_path, codec, data):
    name = str(tmp_path / "seg.mkv")
    tmp = name + "_tmp." + EXT[codec]
    with open(tmp, "wb") as f:
        f.write(data)
    fn = {"h264": framesize.get_framesize_h264, "h265": framesize.get_framesize_h265,
          "vp9": framesize.get_framesize_vp9}[codec]
    buf = io.StringIO()
    try:
        with contextlib.redirect_stdout(buf):
            res = fn(name, False)
    except Exception as e:  # noqa: BLE001
        res = {"error": type(e).__name__, "message": str(e)}
    return {"result": res, "stdout": buf.getvalue(), "removed": not os.path.exists(tmp)}


def expect(case):
    return {k: case[k] for k in ("result", "stdout", "removed")}


def _small():
    return [pytest.param(c, id="%s-%s" % (c["codec"], c["name"])) for c in FX["small"]]


def _medium():
    by = {n: (codec, b) for n, codec, _, b in fs.medium_cases()}
    return [pytest.param(c, by[c["name"]][1], id=c["name"]) for c in FX["medium"]]


def _ivf():
    by = dict(fs.ivf_cases())
    return [pytest.param(c, by[c["name"]], id=c["name"]) for c in FX["ivf"]]


@pytest.mark.parametrize("case", _small())
def test_small_streams_match_reference(tmp_path, case):
    data = base64.b64decode(case["data"])
    assert run_mirror(tmp_path, case["codec"], data) == expect(case)


@pytest.mark.parametrize("case,build", _medium())
def test_medium_streams_match_reference(tmp_path, case, build):
    data = build()
    assert fs.sha256(data) == case["sha256"], "stream builder drifted from the fixture"
    assert run_mirror(tmp_path, case["codec"], data) == expect(case)


@pytest.mark.parametrize("case,build", _ivf())
def test_ivf_streams_match_reference(tmp_path, case, build):
    data = build()
    assert fs.sha256(data) == case["sha256"], "stream builder drifted from the fixture"
    assert run_mirror(tmp_path, "vp9", data) == expect(case)


@pytest.mark.parametrize("case", FX["delete_packets"], ids=lambda c: c["name"])
def test_delete_packets_matches_reference(case):
    lst = copy.deepcopy(case["input"])
    try:
        framesize.delete_packets(lst)
        res = lst
    except Exception as e:  # noqa: BLE001
        res = {"error": type(e).__name__}
    assert res == case["result"]


def test_oracle_pinned_by_fixtures():
    for c in FX["small"]:
        data = base64.b64decode(c["data"])
        try:
            got = ref.annexb_sizes(data, c["codec"])
        except ValueError:
            got = "ValueError"
        want = "ValueError" if isinstance(c["result"], dict) else c["result"]
        assert got == want, c["name"]
    for (name, codec, _, build), c in zip(fs.medium_cases(), FX["medium"]):
        assert ref.annexb_sizes(build(), codec) == c["result"], name
    for (name, build), c in zip(fs.ivf_cases(), FX["ivf"]):
        sizes, mis = ref.ivf_sizes(build())
        assert sizes == c["result"] and c["stdout"].count("\n") == mis, name


def outcome(fn, *a):
    try:
        return fn(*a)
    except ValueError as e:
        return ("ValueError", str(e))


@pytest.mark.parametrize("codec", ["h264", "h265"])
@pytest.mark.parametrize("seed", range(6))
def test_native_scanner_fuzz_vs_oracle(codec, seed):
    rng = np.random.default_rng(1000 + seed)
    alphabets = [[0, 0, 1, 0x65, 0x41, 0x26, 0x02, 0x09], [0, 1, 2, 3, 0x67, 0x81, 0x13, 0x2b, 0x7f],
                 list(range(256))]
    for trial in range(20):
        a = np.array(alphabets[trial % 3], dtype=np.uint8)
        n = int(rng.integers(0, 3000))
        data = a[rng.integers(0, len(a), n)]
        if codec == "h264":  # keep clear of the reference's ValueError bytes except where asked
            bad = ((data & 15) == 1) | ((data & 15) == 5)
            data[bad & (data >= 0xa0)] = 0x65
        assert framesize.annexb_frame_sizes(data, codec) == ref.annexb_sizes(data.tobytes(), codec)
    data = fs.annexb(77 + seed, codec, 400, emulation=bool(seed % 2))  # raw payloads may hit the ValueError
    assert outcome(framesize.annexb_frame_sizes, np.frombuffer(data, np.uint8), codec) == \
        outcome(ref.annexb_sizes, data, codec)


def test_native_valueerror_matches_oracle():
    data = b"\x00\x00\x01\x65\x00\x00\x00\x01\xe1\x00"
    with pytest.raises(ValueError, match="'e'"):
        framesize.annexb_frame_sizes(np.frombuffer(data, np.uint8), "h264")
    with pytest.raises(ValueError, match="'e'"):
        ref.annexb_sizes(data, "h264")


@pytest.mark.parametrize("seed", range(4))
def test_native_ivf_fuzz_vs_oracle(seed):
    rng = np.random.default_rng(seed)
    for trial in range(30):
        data = fs.ivf(int(rng.integers(1 << 30)), int(rng.integers(0, 40)), mean_size=int(rng.integers(1, 200)),
                      bad_marker=float(rng.random()), truncate=int(rng.integers(0, 20)))
        assert framesize.ivf_frame_sizes(np.frombuffer(data, np.uint8)) == ref.ivf_sizes(data)


def test_many_frames_grow_the_output():
    """More frames than the first capacity guess: the scanner is re-run with the count."""
    data = b"\x00\x00\x01\x65" * 5000
    assert framesize.annexb_frame_sizes(np.frombuffer(data, np.uint8), "h264") == ref.annexb_sizes(data, "h264")


@pytest.mark.parametrize("case", FX["convert_file"], ids=lambda c: c["codec"])
def test_convert_file_strings(monkeypatch, case):
    """The remux commands are the reference's (lib/get_framesize.py:54-77)."""
    seen = []
    monkeypatch.setattr(framesize, "run_command", lambda cmd, name="": seen.append([cmd, name]))
    assert framesize.convert_file("/db/segments/a.mp4", case["codec"], case["force"]) == case["return"]
    assert seen == case["commands"]
