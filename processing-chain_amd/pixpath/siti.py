"""P.910 SI/TI behind the reference's SRC-analysis hooks.

Mirrors util/SRC_analysis.py (md5sum :33-43, sum_file :83-104, analyse_src
:120-147) and util/complexity_classification.py (get_difficulty :50-69,
classify_complexity :72-88, encode_file :134-141, main :144-247) with the same
signatures and outputs; SI/TI are ADDED (extra "siti" YAML key / extra `si`,
`ti` CSV columns) and everything else is byte-identical to the reference's
output (pinned by tests/golden/src_analysis_fixtures.json).  The per-frame SI/TI runs on the MI355X
(pp_siti, spec PP-SITI-1) over decoded luma batches; frame ranges of one SRC
can be split across GPUs with a one-frame halo (``prev``).
"""
import hashlib
import io
import json
import math
import os
import subprocess

import numpy as np

REFERENCE_BITRATE = 2.75  # complexity_classification.py:34
DIFFICULTY_CLASS_THRESHOLDS = [[6, 4], [7, 6], [8, 8]]


# ---------------------------------------------------------------- SRC_analysis
def md5sum(src, ordernum, length=io.DEFAULT_BUFFER_SIZE):
    """util/SRC_analysis.py:33-43 (prints the same progress line)."""
    md5 = hashlib.md5()
    with io.open(src, mode="rb") as fd:
        for chunk in iter(lambda: fd.read(length), b""):
            md5.update(chunk)
    print("#{} is done, name: {}".format(str(ordernum).zfill(2), os.path.basename(src)))
    return md5


def sum_file(videofile, ordernum):
    """util/SRC_analysis.py:83-104: verify or write <file>.md5."""
    base = os.path.basename(videofile)
    md5file = os.path.abspath(videofile) + ".md5"
    existing = None
    if os.path.isfile(md5file):
        with open(md5file) as f:
            existing = f.readlines()[0].strip().split(" ")[0]
    cur = md5sum(videofile, ordernum)
    if existing:
        if existing == cur.hexdigest():
            return "ok    -- File: {} has a correct md5sum".format(base)
        return "BAD!! -- File: {} has an erroneous md5sum".format(base)
    with open(md5file, "w+") as f:
        f.write(str(cur.hexdigest()) + " " + base + "\n")
    return "md5sum file written for file: {}".format(base)


def siti_of_batch(luma, bitdepth, prev=None):
    """Per-frame SI/TI (numpy float64 arrays) of a [N, H, W] luma batch on the GPU.
    ``luma`` may be a numpy array or a (device) torch tensor."""
    import torch

    from . import ops
    t = luma if isinstance(luma, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(luma))
    if t.device.type != "cuda":
        t = t.cuda()
    p = None
    if prev is not None:
        p = prev if isinstance(prev, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(prev))
        p = p.to(t.device)
    si, ti = ops.siti(t, bitdepth, prev=p)
    torch.cuda.current_stream(t.device).synchronize()
    return si.cpu().numpy(), ti.cpu().numpy()


def siti_summary(si, ti):
    """(SI, TI) = max over frames (TI ignores its undefined first frame)."""
    ti = np.asarray(ti, dtype=np.float64)
    ti = ti[~np.isnan(ti)]
    return float(np.max(si)) if len(si) else float("nan"), float(np.max(ti)) if ti.size else float("nan")


def siti_of_file(videofile, batch=120, reader=None):
    """Decode a file (ffmpeg, or y4m/raw via pixpath.io) and return per-frame SI/TI."""
    from . import io as pio
    rd = reader or pio.open_reader(videofile)
    sis, tis, prev = [], [], None
    for frames in rd.batches(batch):
        luma = frames[0]
        si, ti = siti_of_batch(luma, rd.fmt.depth, prev=prev)
        sis.append(si)
        tis.append(ti)
        prev = luma[-1]
    rd.close()
    return np.concatenate(sis), np.concatenate(tis)


def siti_yaml_entry(si, ti):
    """The extra "siti" key of <src>.yaml (spec PP-SITI-1)."""
    SI, TI = siti_summary(si, ti)
    return {"si": SI, "ti": TI, "si_frames": [float(v) for v in si],
            "ti_frames": [None if math.isnan(v) else float(v) for v in ti],
            "spec": "PP-SITI-1 (ITU-T P.910 Sobel/frame-difference, valid-region SI, ddof=0)"}


def analyse_src(videofile, ordernum, with_siti=True, src_info=None, stream_sizes=None, reader=None, siti=None):
    """util/SRC_analysis.py:120-147 plus an extra "siti" key.

    get_src_info / get_stream_size go through ffprobe exactly as the
    reference's (pixpath.probe); the keys the reference writes come out
    byte-identical (tests/test_src_analysis_parity.py).  ``src_info`` /
    ``stream_sizes`` replace those probes, ``reader`` the decode for SI/TI
    (pixpath.io reader), ``siti`` precomputed (si_frames, ti_frames)."""
    import yaml
    from . import probe
    videoinfo = src_info if src_info is not None else probe.get_src_info(videofile)
    if stream_sizes is None:
        stream_sizes = {"v": probe.get_stream_size(videofile), "a": probe.get_stream_size(videofile, "audio")}
    md5filename = videofile + ".md5"
    if not os.path.isfile(md5filename):
        md5hash = str(md5sum(videofile, ordernum).hexdigest())
    else:
        with open(md5filename) as f:
            md5hash = f.readlines()[0].strip().split(" ")[0]
    ret = {"md5sum": md5hash, "get_stream_size": {"v": stream_sizes["v"], "a": stream_sizes["a"]},
           "get_src_info": videoinfo}
    if with_siti:
        si, ti = siti if siti is not None else siti_of_file(videofile, reader=reader)
        ret["siti"] = siti_yaml_entry(si, ti)
    yaml_path = videofile + ".yaml"
    with open(yaml_path, "w") as outfile:
        yaml.dump(ret, outfile, default_flow_style=False)
    return yaml_path


# ------------------------------------------------------ complexity_classification
def difficulty_from_info(output_file, info):
    """The get_difficulty formula (util/complexity_classification.py:50-69) on a
    get_segment_info()-shaped dict."""
    size = info["file_size"]
    duration = info["video_duration"]
    framerate = info["video_frame_rate"]
    nr_pixels = info["video_width"] * info["video_height"]
    norm_bitrate = size / framerate / duration / (nr_pixels / 1000)
    return {
        "file": os.path.basename(output_file),
        "norm_bitrate": norm_bitrate,
        "complexity": 20 * math.log(norm_bitrate, 10) / REFERENCE_BITRATE,
        "framerate": float(framerate),
        "width": int(info["video_width"]),
        "height": int(info["video_height"]),
        "size": int(size),
        "duration": float(duration),
    }


def get_difficulty(output_file):
    """util/complexity_classification.py:50-69 (get_segment_info through ffprobe, pixpath.probe)."""
    from . import probe
    return difficulty_from_info(output_file, probe.get_segment_info(output_file))


def classify_complexity(complexity, framerate, quantiles):
    """util/complexity_classification.py:72-88."""
    q = quantiles["low"] if framerate <= 30 else quantiles["high"]
    if complexity > q[0.50]:
        return 3 if complexity > q[0.75] else 2
    return 1 if complexity > q[0.25] else 0


def encode_file(input_file, output_file):
    """util/complexity_classification.py:134-141 (CRF-23 x264 encode command)."""
    return ("ffmpeg -nostdin -y -i '{input_file}' -pix_fmt yuv420p -an -c:v libx264 -crf 23 "
            "'{output_file}'").format(**locals())


def add_siti_columns(rows, siti_by_file):
    """Extra CSV columns `si`, `ti` for the complexity table (the consumer,
    reference lib/test_config.py:1250-1257, reads only file/complexity_class)."""
    out = []
    for r in rows:
        r = dict(r)
        si, ti = siti_by_file.get(r["file"], (float("nan"), float("nan")))
        r["si"], r["ti"] = si, ti
        out.append(r)
    return out


def siti_from_yaml(src_file):
    """(SI, TI) from <src>.yaml written by analyse_src, or None."""
    import yaml
    p = src_file + ".yaml"
    if not os.path.isfile(p):
        return None
    with open(p) as f:
        d = yaml.safe_load(f) or {}
    e = d.get("siti")
    return (float(e["si"]), float(e["ti"])) if e else None


def complexity_parse_args(argv=None):
    """util/complexity_classification.py:91-131, plus --siti {yaml,gpu,none}."""
    import argparse
    ap = argparse.ArgumentParser(description="Complexity classification",
                                 formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    ap.add_argument("-i", "--input", required=True, nargs="+", help="Input files (SRCs)")
    ap.add_argument("-t", "--tmp-dir", default=os.path.join(os.getcwd(), "complexityAnalysis"),
                    help="Path to (temporary) complexity analysis folder")
    ap.add_argument("-p", "--parallelism", default=1, help="Number of parallel encodes")
    ap.add_argument("-o", "--output-file", default="complexity_classification.csv", help="Filename of CSV output file")
    ap.add_argument("-f", "--force", action="store_true", help="Force overwriting (re-analyzing) existing files")
    ap.add_argument("-v", "--verbose", action="store_true", help="Print debug messages")
    ap.add_argument("-n", "--dry-run", action="store_true", help="Show what would be run instead of running it")
    ap.add_argument("--siti", default="yaml", choices=["yaml", "gpu", "none"],
                    help="si/ti columns: from <src>.yaml (analyse_src), measured on the GPU when absent, or left out")
    return ap.parse_args(argv)


def complexity_main(argv=None):
    """util/complexity_classification.py:144-247 with `si`, `ti` columns appended
    (SI/TI of each SRC: its <src>.yaml from analyse_src, else -- with --siti gpu --
    measured on the MI355X).  Without them the CSV is byte-identical to the
    reference's (tests/test_src_analysis_parity.py)."""
    import logging
    import subprocess
    import sys
    from multiprocessing import Pool

    import pandas as pd
    log = logging.getLogger("main")
    a = complexity_parse_args(argv)
    if a.verbose:
        log.setLevel(logging.DEBUG)
    if not os.path.isdir(a.tmp_dir):
        log.info("temporary directory " + str(a.tmp_dir) + " does not exist, creating")
        os.mkdir(a.tmp_dir)
    if not a.output_file.endswith(".csv"):
        log.error("Output file must be .csv!")
        sys.exit(1)
    input_files = [f for f in a.input if f.endswith(".avi")]
    cmds, outputs, src_of = [], [], {}
    for input_file in input_files:
        base = os.path.splitext(os.path.basename(input_file))[0]
        output_file = os.path.join(a.tmp_dir, base + "_crf23.avi")
        if not (os.path.isfile(output_file) and not a.force):
            if encode_file(input_file, output_file) not in cmds:  # ParallelRunner keeps a set
                cmds.append(encode_file(input_file, output_file))
        outputs.append(output_file)
        src_of[os.path.basename(output_file)] = input_file
    if a.dry_run:
        for c in cmds:
            log.info(c)
        sys.exit(0)
    if cmds:
        with Pool(int(a.parallelism)) as pool:
            rcs = pool.map(_shell_rc, cmds)
        if any(rcs):
            log.error("There were errors in your commands. Please check the output and re-run the processing chain!")
            sys.exit(1)
    all_data = [get_difficulty(o) for o in outputs]
    if not all_data:
        log.error("No info calculated, exiting")
        sys.exit(1)
    df = pd.DataFrame(all_data)[["file", "norm_bitrate", "complexity", "framerate", "width", "height", "size",
                                 "duration"]].sort_values("file")
    quants = {"low": df[df["framerate"] <= 30]["complexity"].quantile([0.25, 0.5, 0.75]),
              "high": df[df["framerate"] > 30]["complexity"].quantile([0.25, 0.5, 0.75])}
    df["complexity_class"] = df.apply(lambda x: classify_complexity(x["complexity"], x["framerate"], quants), axis=1)
    if a.siti != "none":
        vals = {}
        for f in df["file"]:
            src = src_of[f]
            v = siti_from_yaml(src)
            if v is None and a.siti == "gpu":
                v = siti_summary(*siti_of_file(src))
            vals[f] = v if v is not None else (float("nan"), float("nan"))
        df["si"] = [vals[f][0] for f in df["file"]]
        df["ti"] = [vals[f][1] for f in df["file"]]
    csv_file = os.path.join(a.tmp_dir, a.output_file)
    log.info("Writing complexity data to " + str(csv_file))
    df.to_csv(csv_file, index=False)
    return csv_file


def _shell_rc(cmd):
    import subprocess
    return subprocess.run(cmd, shell=True).returncode


def dump_json(obj, path):
    with open(path, "w") as f:
        json.dump(obj, f, indent=1)


def _ffprobe_json(path):  # pragma: no cover - needs ffprobe
    out = subprocess.run(["ffprobe", "-loglevel", "error", "-show_streams", "-of", "json", path],
                         check=True, capture_output=True).stdout
    return json.loads(out)
