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


def siti_of_batch(luma, bitdepth, prev=None, normalize=False):
    """Per-frame SI/TI (numpy float64 arrays) of a [N, H, W] luma batch on the GPU.
    ``luma`` may be a numpy array or a (device) torch tensor.  ``normalize``:
    values on the 8-bit scale (divided by 2^(bitdepth-8), PP_SITI_NORMALIZE)."""
    import torch

    from . import ops
    t = luma if isinstance(luma, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(luma))
    if t.device.type != "cuda":
        t = t.cuda()
    p = None
    if prev is not None:
        p = prev if isinstance(prev, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(prev))
        p = p.to(t.device)
    si, ti = ops.siti(t, bitdepth, prev=p, normalize=normalize)
    torch.cuda.current_stream(t.device).synchronize()
    return si.cpu().numpy(), ti.cpu().numpy()


def siti_summary(si, ti):
    """(SI, TI) = max over frames (TI ignores its undefined first frame)."""
    ti = np.asarray(ti, dtype=np.float64)
    ti = ti[~np.isnan(ti)]
    return float(np.max(si)) if len(si) else float("nan"), float(np.max(ti)) if ti.size else float("nan")


def siti_of_file(videofile, batch=120, reader=None, normalize=False, with_depth=False):
    """Per-frame SI/TI of a file: decoded luma only (pixpath.io.LumaReader:
    y4m/raw seek past chroma, ffmpeg decodes to gray/gray10le), streamed
    through pinned double buffers (siti_stream).  ``reader``: a full-frame
    pixpath.io reader instead (its luma plane is used).  Returns (si, ti) or,
    with_depth, (si, ti, bitdepth)."""
    from . import io as pio
    if reader is not None:
        rd = _LumaOf(reader)
    else:
        rd = pio.LumaReader(videofile)
    try:
        si, ti = siti_stream(rd, batch=batch, normalize=normalize)
    finally:
        rd.close()
    return (si, ti, rd.depth) if with_depth else (si, ti)


class _LumaOf:
    """A full-frame pixpath.io reader seen as a luma reader."""

    def __init__(self, rd):
        self.rd, self.w, self.h, self.depth = rd, rd.w, rd.h, rd.fmt.depth
        self.luma_bytes = self.w * self.h * (2 if self.depth > 8 else 1)
        self._buf = None

    def read_into(self, buf, n):
        fb = self.rd.frame_bytes
        if self._buf is None or len(self._buf) < n * fb:
            self._buf = np.empty(n * fb, np.uint8)
        k = self.rd.read_into(self._buf, n)
        out = np.frombuffer(memoryview(buf).cast("B"), np.uint8)
        lb = self.luma_bytes
        for i in range(k):
            out[i * lb:(i + 1) * lb] = self._buf[i * fb:i * fb + lb]
        return k

    def close(self):
        self.rd.close()


def siti_stream(rd, batch=120, normalize=False, device=None):
    """SI/TI of every frame a luma reader yields, with the host read, the H2D
    copy and the kernel of neighbouring batches overlapped: a reader thread
    fills pinned buffers, H2D runs on a copy stream into one of three device
    slots, pp_siti on a compute stream with the previous batch's last frame
    (still resident in its slot) as the TI halo.  Slot k+1's H2D waits for
    batch k-1's kernel (the last reader of that slot)."""
    import queue
    import threading

    import torch

    from . import ops
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    B, lb = int(batch), rd.luma_bytes
    dt = torch.uint16 if rd.depth > 8 else torch.uint8
    h_in = [torch.empty((B, lb), dtype=torch.uint8).pin_memory() for _ in range(2)]
    d_in = [torch.empty((B, rd.h, rd.w), dtype=dt, device=dev) for _ in range(3)]
    copy_s, comp_s = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    comp_done = [None, None, None]
    free_in, rq, err = queue.Queue(), queue.Queue(maxsize=2), []
    for i in range(2):
        free_in.put(i)

    def read_loop():
        try:
            while True:
                slot = free_in.get()
                n = rd.read_into(h_in[slot].numpy(), B)
                rq.put((slot, n))
                if n < B:
                    return
        except Exception as e:  # surfaced in the caller's thread
            err.append(e)
            rq.put((None, 0))

    th = threading.Thread(target=read_loop, daemon=True)
    th.start()
    outs, prev, k = [], None, 0
    while True:
        slot, n = rq.get()
        if slot is None or n == 0:
            break
        ds = k % 3
        with torch.cuda.stream(copy_s):
            if comp_done[(k + 1) % 3] is not None:  # batch k-2 read slot ds (k-1 used it as halo: waited below)
                copy_s.wait_event(comp_done[(k + 1) % 3])
            if comp_done[ds] is not None:
                copy_s.wait_event(comp_done[ds])
            d_in[ds].view(torch.uint8).view(B, lb)[:n].copy_(h_in[slot][:n], non_blocking=True)
            h2d = torch.cuda.Event()
            h2d.record(copy_s)
        comp_s.wait_event(h2d)
        with torch.cuda.stream(comp_s):
            si, ti = ops.siti(d_in[ds][:n], rd.depth, prev=prev, stream=comp_s, normalize=normalize)
            ev = torch.cuda.Event()
            ev.record(comp_s)
        comp_done[ds] = ev
        outs.append((si, ti))
        prev = d_in[ds][n - 1]
        h2d.synchronize()  # the pinned buffer is free again
        free_in.put(slot)
        k += 1
        if n < B:
            break
    th.join(timeout=5.0)
    if err:
        raise err[0]
    comp_s.synchronize()
    if not outs:
        return np.zeros(0), np.zeros(0)
    return (torch.cat([o[0] for o in outs]).cpu().numpy(), torch.cat([o[1] for o in outs]).cpu().numpy())


def siti_scale(bitdepth, normalize):
    """Factor applied to the raw-code-value SI/TI: 1, or 2^-(bitdepth-8) when normalised."""
    return 1.0 / (1 << (int(bitdepth) - 8)) if normalize else 1.0


def siti_yaml_entry(si, ti, bitdepth=None, normalize=False):
    """The extra "siti" key of <src>.yaml (spec PP-SITI-1).  ``bitdepth`` and
    ``scale`` record the SRC's luma depth and the factor applied to the raw
    code values (1, or 2^-(bitdepth-8) with the 8-bit-scale normalisation),
    so 8- and 10-bit SRCs can be compared."""
    SI, TI = siti_summary(si, ti)
    e = {"si": SI, "ti": TI, "si_frames": [float(v) for v in si],
         "ti_frames": [None if math.isnan(v) else float(v) for v in ti],
         "spec": "PP-SITI-1 (ITU-T P.910 Sobel/frame-difference, valid-region SI, ddof=0)"}
    if bitdepth is not None:
        e["bitdepth"] = int(bitdepth)
        e["scale"] = siti_scale(bitdepth, normalize)
        e["normalized"] = bool(normalize)
    return e


def analyse_src(videofile, ordernum, with_siti=True, src_info=None, stream_sizes=None, reader=None, siti=None,
                normalize=False, bitdepth=None):
    """util/SRC_analysis.py:120-147 plus an extra "siti" key.

    get_src_info / get_stream_size go through ffprobe exactly as the
    reference's (pixpath.probe); the keys the reference writes come out
    byte-identical (tests/test_src_analysis_parity.py).  ``src_info`` /
    ``stream_sizes`` replace those probes, ``reader`` the decode for SI/TI
    (pixpath.io reader), ``siti`` precomputed (si_frames, ti_frames) of a
    ``bitdepth``-bit SRC; ``normalize`` puts SI/TI on the 8-bit scale."""
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
        if siti is not None:
            si, ti = siti
        else:
            si, ti, bitdepth = siti_of_file(videofile, reader=reader, normalize=normalize, with_depth=True)
        ret["siti"] = siti_yaml_entry(si, ti, bitdepth, normalize)
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


def siti_from_yaml(src_file, with_depth=False):
    """(SI, TI) from <src>.yaml written by analyse_src, or None; with_depth:
    (SI, TI, bitdepth, scale) -- bitdepth None and scale 1.0 for entries
    written without them."""
    import yaml
    p = src_file + ".yaml"
    if not os.path.isfile(p):
        return None
    with open(p) as f:
        d = yaml.safe_load(f) or {}
    e = d.get("siti")
    if not e:
        return None
    if with_depth:
        return float(e["si"]), float(e["ti"]), e.get("bitdepth"), float(e.get("scale", 1.0))
    return float(e["si"]), float(e["ti"])


def _script_dir():
    """The directory of the running script (the reference's
    util/complexity_classification.py when it calls complexity_main, as
    INTEGRATION.md section 4 wires it), else the working directory."""
    import sys
    f = getattr(sys.modules.get("__main__"), "__file__", None)
    return os.path.dirname(os.path.abspath(f)) if f else os.getcwd()


def complexity_parse_args(argv=None, script_dir=None):
    """util/complexity_classification.py:91-131, plus --siti {yaml,gpu,none}.
    --tmp-dir defaults to `complexityAnalysis` next to the script, as the
    reference's (:100-105: os.path.dirname(os.path.abspath(__file__)));
    script_dir overrides which script that is."""
    import argparse
    ap = argparse.ArgumentParser(description="Complexity classification",
                                 formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    ap.add_argument("-i", "--input", required=True, nargs="+", help="Input files (SRCs)")
    ap.add_argument("-t", "--tmp-dir", default=os.path.join(script_dir or _script_dir(), "complexityAnalysis"),
                    help="Path to (temporary) complexity analysis folder")
    ap.add_argument("-p", "--parallelism", default=1, help="Number of parallel encodes")
    ap.add_argument("-o", "--output-file", default="complexity_classification.csv", help="Filename of CSV output file")
    ap.add_argument("-f", "--force", action="store_true", help="Force overwriting (re-analyzing) existing files")
    ap.add_argument("-v", "--verbose", action="store_true", help="Print debug messages")
    ap.add_argument("-n", "--dry-run", action="store_true", help="Show what would be run instead of running it")
    ap.add_argument("--siti", default="yaml", choices=["yaml", "gpu", "none"],
                    help="si/ti columns: from <src>.yaml (analyse_src), measured on the GPU when absent, or left out")
    ap.add_argument("--siti-scale", default="native", choices=["native", "8bit"],
                    help="si/ti in raw code values of each SRC's bit depth, or all on the 8-bit scale "
                         "(divided by 2^(bitdepth-8))")
    return ap.parse_args(argv)


def complexity_main(argv=None, script_dir=None):
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
    a = complexity_parse_args(argv, script_dir)
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
        # si, ti plus the SRC's luma bit depth and the factor applied to its raw
        # code values (1 native; 2^-(bitdepth-8) on the 8-bit scale)
        norm = a.siti_scale == "8bit"
        vals = {}
        for f in df["file"]:
            src = src_of[f]
            v = siti_from_yaml(src, with_depth=True)
            if v is not None and norm and v[2] is not None and v[3] == 1.0:  # raw YAML values -> 8-bit scale
                k = siti_scale(v[2], True)
                v = (v[0] * k, v[1] * k, v[2], k)
            elif v is not None and not norm and v[2] is not None and v[3] != 1.0:  # normalised YAML -> raw
                v = (v[0] / v[3], v[1] / v[3], v[2], 1.0)
            if v is None and a.siti == "gpu":
                si_f, ti_f, depth = siti_of_file(src, normalize=norm, with_depth=True)
                v = siti_summary(si_f, ti_f) + (depth, siti_scale(depth, norm))
            vals[f] = v if v is not None else (float("nan"), float("nan"), None, float("nan"))
        df["si"] = [vals[f][0] for f in df["file"]]
        df["ti"] = [vals[f][1] for f in df["file"]]
        df["siti_bitdepth"] = pd.array([vals[f][2] for f in df["file"]], dtype="Int64")
        df["siti_scale"] = [vals[f][3] for f in df["file"]]
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
