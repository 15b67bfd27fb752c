#!/usr/bin/env python3
"""A stand-in `ffprobe` for fixture generation and CPU tests (SURVEY.md section 4,
"fake-backend technique").  It answers the three ffprobe command shapes the
reference's lib/ffmpeg.py issues -- and that pixpath.io mirrors -- from canned
JSON, keyed by the probed file's basename:

  -select_streams v -show_streams -of json FILE          (get_src_info, :600)
  -show_streams -of json FILE                            (get_segment_info, :459)
  -select_streams v|a -show_entries packet=size -of compact=p=0:nk=1 FILE
                                                         (get_stream_size, :406)
  -select_streams v -show_packets -show_entries ... -of json FILE
                                                         (get_segment_info fallback, :487)

The database is the JSON file named by $FAKE_FFPROBE_DB:
  {basename: {"streams": [...], "packets": {"v": [sizes], "a": [sizes]},
              "vfi": [packet dicts]}}
An unknown file exits 1 with ffprobe's message, like the real tool.
"""
import json
import os
import sys


def main(argv):
    db = json.load(open(os.environ["FAKE_FFPROBE_DB"]))
    path = argv[-1]
    entry = db.get(os.path.basename(path))
    if entry is None or not os.path.exists(path):
        sys.stderr.write("%s: No such file or directory\n" % path)
        return 1
    sel = None
    if "-select_streams" in argv:
        sel = argv[argv.index("-select_streams") + 1]
    kind = {"v": "video", "a": "audio"}.get(sel)
    if "-show_packets" in argv:
        sys.stdout.write(json.dumps({"packets": entry.get("vfi", [])}, indent=4) + "\n")
    elif "-show_streams" in argv:
        streams = [s for s in entry["streams"] if kind is None or s.get("codec_type") == kind]
        sys.stdout.write(json.dumps({"streams": streams}, indent=4) + "\n")
    elif "-show_entries" in argv and argv[argv.index("-show_entries") + 1] == "packet=size":
        for s in entry.get("packets", {}).get(sel, []):
            sys.stdout.write("%d\n" % s)
    else:
        sys.stderr.write("fake ffprobe: unsupported arguments %r\n" % (argv,))
        return 2
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
