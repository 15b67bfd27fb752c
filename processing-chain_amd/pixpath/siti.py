"""P.910 SI/TI behind the reference's SRC-analysis hooks.

Mirrors util/SRC_analysis.py (md5sum :33-43, sum_file :83-104, analyse_src
:120-147) and util/complexity_classification.py (get_difficulty :50-69,
classify_complexity :72-88, encode_file :134-141) with the same signatures and
outputs; SI/TI are ADDED (extra "siti" YAML key / extra CSV columns) and the
existing keys stay byte-identical.  The per-frame SI/TI runs on the MI355X
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


def analyse_src(videofile, ordernum, with_siti=True, src_info=None, stream_sizes=None):
    """util/SRC_analysis.py:120-147 plus an extra "siti" key.

    The reference fills get_src_info/get_stream_size by ffprobe
    (lib/ffmpeg.py:566-633, :399-417); those probes are passed in
    (``src_info``, ``stream_sizes``) or taken from pixpath.io.probe()."""
    import yaml
    from . import io as pio
    if src_info is None or stream_sizes is None:
        pr = pio.probe(videofile)
        src_info = src_info if src_info is not None else pr["stream"]
        stream_sizes = stream_sizes if stream_sizes is not None else pr["sizes"]
    md5filename = videofile + ".md5"
    if not os.path.isfile(md5filename):
        md5hash = str(md5sum(videofile, ordernum).hexdigest())
    else:
        with open(md5filename) as f:
            md5hash = f.readlines()[0].strip().split(" ")[0]
    ret = {"md5sum": md5hash, "get_stream_size": {"v": stream_sizes["v"], "a": stream_sizes["a"]},
           "get_src_info": src_info}
    if with_siti:
        si, ti = siti_of_file(videofile)
        SI, TI = siti_summary(si, ti)
        ret["siti"] = {"si": SI, "ti": TI, "si_frames": [float(v) for v in si],
                       "ti_frames": [None if math.isnan(v) else float(v) for v in ti],
                       "spec": "PP-SITI-1 (ITU-T P.910 Sobel/frame-difference, valid-region SI, ddof=0)"}
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
    """util/complexity_classification.py:50-69 (probe through ffprobe)."""
    from . import io as pio
    return difficulty_from_info(output_file, pio.segment_info(output_file))


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


def dump_json(obj, path):
    with open(path, "w") as f:
        json.dump(obj, f, indent=1)


def _ffprobe_json(path):  # pragma: no cover - needs ffprobe
    out = subprocess.run(["ffprobe", "-loglevel", "error", "-show_streams", "-of", "json", path],
                         check=True, capture_output=True).stdout
    return json.loads(out)
