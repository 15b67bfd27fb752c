#!/usr/bin/env python3
"""Generate tests/golden/framesize_fixtures.json by running the REFERENCE's own
p02 scanners (lib/get_framesize.py, read-only at $REFERENCE, default
/root/reference) on the synthetic streams of tests/framesize_streams.py.

Build container only (the reference does not travel to the GPU box).  Each
stream is written to <tmp>/seg.mkv_tmp.<ext> and the reference function is
called with force=False, so its convert_file() returns that file without
running ffmpeg (lib/get_framesize.py:72-74); the scanner then reads and removes
it.  Recorded: the returned sizes (or the exception type and message), what it
printed, and whether the temp file was removed.  delete_packets
(lib/get_framesize.py:27-51) is recorded as the list it leaves behind.

Reference functions exercised (file:line):
  lib/get_framesize.py:27   delete_packets
  lib/get_framesize.py:87   get_framesize_vp9
  lib/get_framesize.py:144  get_framesize_h264
  lib/get_framesize.py:204  get_framesize_h265
"""
import base64
import contextlib
import copy
import io
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))  # tests/
REFERENCE = os.environ.get("REFERENCE", "/root/reference")

import framesize_streams as fs  # noqa: E402

EXT = {"h264": "h264", "h265": "h265", "vp9": "ivf"}


def run_ref(gf, codec, data):
    fn = {"h264": gf.get_framesize_h264, "h265": gf.get_framesize_h265, "vp9": gf.get_framesize_vp9}[codec]
    with tempfile.TemporaryDirectory() as d:
        name = os.path.join(d, "seg.mkv")
        tmp = name + "_tmp." + EXT[codec]
        with open(tmp, "wb") as f:
            f.write(data)
        buf = io.StringIO()
        try:
            with contextlib.redirect_stdout(buf):
                res = fn(name, False)
        except Exception as e:  # noqa: BLE001 -- the reference's own failure, recorded as data
            res = {"error": type(e).__name__, "message": str(e)}
        return {"result": res, "stdout": buf.getvalue(), "removed": not os.path.exists(tmp)}


def main():
    sys.path.insert(0, REFERENCE)
    import lib.get_framesize as gf

    out = {"generator": "tests/golden/gen_framesize_fixtures.py", "reference": "lib/get_framesize.py",
           "small": [], "medium": [], "ivf": [], "delete_packets": []}
    for name, codec, data in fs.small_cases():
        out["small"].append({"name": name, "codec": codec, "data": base64.b64encode(data).decode(),
                             **run_ref(gf, codec, data)})
    for codec in ("h264", "h265"):
        out["small"].append({"name": "empty", "codec": codec, "data": "", **run_ref(gf, codec, b"")})
    for name, codec, seed, build in fs.medium_cases():
        data = build()
        out["medium"].append({"name": name, "codec": codec, "seed": seed, "bytes": len(data),
                              "sha256": fs.sha256(data), **run_ref(gf, codec, data)})
    for name, build in fs.ivf_cases():
        data = build()
        out["ivf"].append({"name": name, "bytes": len(data), "sha256": fs.sha256(data), **run_ref(gf, "vp9", data)})
    for name, vfi in fs.vfi_cases():
        lst = copy.deepcopy(vfi)
        try:
            gf.delete_packets(lst)
            res = lst
        except Exception as e:  # noqa: BLE001
            res = {"error": type(e).__name__}
        out["delete_packets"].append({"name": name, "input": vfi, "result": res})

    # convert_file's remux commands (lib/get_framesize.py:54-77), ffmpeg not run
    seen = []
    real = gf.cmd_utils.run_command
    gf.cmd_utils.run_command = lambda cmd, name="": seen.append([cmd, name])
    conv = []
    for codec, force in (("vp9", True), ("h264", False), ("hevc", True), ("h265", False)):
        seen.clear()
        ret = gf.convert_file("/db/segments/a.mp4", codec, force)
        conv.append({"codec": codec, "force": force, "return": ret, "commands": list(seen)})
    gf.cmd_utils.run_command = real
    out["convert_file"] = conv

    path = os.path.join(HERE, "framesize_fixtures.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", path, {k: len(v) for k, v in out.items() if isinstance(v, list)})


if __name__ == "__main__":
    main()
