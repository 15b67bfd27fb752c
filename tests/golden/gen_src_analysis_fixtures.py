#!/usr/bin/env python3
"""Generate tests/golden/src_analysis_fixtures.json by running the REFERENCE's own
Python (read-only at $REFERENCE, default /root/reference) on the synthetic
files of tests/golden/src_scenarios.py, with tests/golden/fake_ffprobe.py as
`ffprobe` on PATH (the SURVEY.md section 4 fake-backend technique).  Only run
in the build container; the JSON is data (inputs and the reference's outputs:
YAML text, segment-info dicts, CSV text), no reference source.

Reference functions exercised (file:line):
  util/SRC_analysis.py:120   analyse_src      -> <src>.yaml text (+ its stdout line)
  lib/ffmpeg.py:566          get_src_info     (r_frame_rate -> str(int(eval(..))), :616-617)
  lib/ffmpeg.py:399          get_stream_size  (reads <file>.yaml when present, :409-412)
  lib/ffmpeg.py:433          get_segment_info (duration from stream / tags / packets, :479-502)
  util/complexity_classification.py:144  main -> complexity CSV text

Quirk recorded, not mirrored: analyse_src passes a Src whose info_path is
False, so get_src_info stats and writes file descriptor 0 (open(False, 'w'),
lib/ffmpeg.py:603, :629): under a terminal it prints a second YAML there.
The generator gives the reference a pseudo-terminal as stdin and records what
it wrote ("fd0_yaml").
"""
import json
import os
import pty
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REFERENCE = os.environ.get("REFERENCE", "/root/reference")
sys.path.insert(0, HERE)
import src_scenarios as sc  # noqa: E402


def inner(root, what):
    sys.path.insert(0, REFERENCE)
    sys.path.insert(0, os.path.join(REFERENCE, "util"))
    import lib.ffmpeg as rff
    out = {}
    if what.startswith("src:"):
        # one analyse_src per process: its get_src_info closes file descriptor 0
        # (with open(False, 'w'), lib/ffmpeg.py:627), so a second call in the
        # same process fails with EBADF -- the reference's single-process loop
        # (SRC_analysis.py:195-199, --concurrency 1) cannot analyse two files
        import contextlib
        import io
        import SRC_analysis as rsa
        _, name, i = what.split(":")
        path = os.path.join(root, name)
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            yp = rsa.analyse_src(path, int(i))
        out = {"ordernum": int(i), "yaml_path_suffix": os.path.relpath(yp, root), "yaml": open(yp).read(),
               "stdout": buf.getvalue()}
    else:
        import complexity_classification as rcc

        class Seg:
            def __init__(self, p):
                self.filename = "random"
                self.file_path = p

            def __str__(self):
                return self.file_path
        out["get_segment_info"] = {}
        for name in sorted(sc.SEGMENTS):
            try:
                r = rff.get_segment_info(Seg(os.path.join(root, name)))
                r = {"ok": [[k, v] for k, v in r.items()]}
            except SystemExit as e:
                r = {"sys_exit": e.code}
            out["get_segment_info"][name] = r
        sys.argv = ["complexity_classification.py", "-i"] + [os.path.join(root, f) for f in sc.COMPLEXITY_INPUTS] + \
            ["-t", os.path.join(root, "complexity"), "-o", "complexity.csv"]
        rcc.main()
        out["complexity_csv"] = open(os.path.join(root, "complexity", "complexity.csv")).read()
    json.dump(out, open(os.path.join(root, "result.json"), "w"))


def run_inner(root, env, what):
    """Run one reference step in a child whose stdin is a fresh pseudo-terminal;
    returns (its result, what it wrote to file descriptor 0)."""
    master, slave = pty.openpty()
    p = subprocess.run([sys.executable, os.path.abspath(__file__), "--inner", root, what], env=env, cwd=root,
                       stdin=slave, capture_output=True, text=True)
    os.close(slave)
    fd0 = b""
    os.set_blocking(master, False)
    try:
        while True:
            chunk = os.read(master, 65536)
            if not chunk:
                break
            fd0 += chunk
    except (BlockingIOError, OSError):
        pass
    os.close(master)
    if p.returncode:
        sys.stderr.write(p.stdout + p.stderr)
        raise SystemExit("reference run failed: " + what)
    return json.load(open(os.path.join(root, "result.json"))), fd0.decode(errors="replace").replace("\r\n", "\n")


def main():
    res = {"analyse_src": {}, "fd0_yaml": {}}
    with tempfile.TemporaryDirectory() as root:
        db = sc.materialise(root)
        env = dict(os.environ, FAKE_FFPROBE_DB=db, PATH=sc.fake_ffprobe_dir(root) + os.pathsep + os.environ["PATH"])
        for i, name in enumerate(sorted(sc.SRC)):
            r, fd0 = run_inner(root, env, "src:%s:%d" % (name, i))
            res["analyse_src"][name] = r
            res["fd0_yaml"][name] = fd0
        r, _ = run_inner(root, env, "segments")
        res.update(r)
    res["generator"] = "tests/golden/gen_src_analysis_fixtures.py"
    res["reference"] = "pnats2avhd/processing-chain 1.0.0"
    path = os.path.join(HERE, "src_analysis_fixtures.json")
    json.dump(res, open(path, "w"), indent=1, sort_keys=True)
    print("wrote", path, "analyse_src:", len(res["analyse_src"]), "segments:", len(res["get_segment_info"]))


if __name__ == "__main__":
    if len(sys.argv) > 3 and sys.argv[1] == "--inner":
        inner(sys.argv[2], sys.argv[3])
    else:
        main()
