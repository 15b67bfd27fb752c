"""`python -m pixpath.cli` -- the GPU-backend commands that pixpath.ffmpeg's
builders return (same positional output file, -y/-n overwrite convention as
the ffmpeg strings they replace).

  encseg p01 encode_segment: trimmed decode -> scale=W:-2 (+ -pix_fmt) -> select/fps -> Y4M
         for the encoder (lib/ffmpeg.py:772-937)
  avpvs  decode -> scale (+ -pix_fmt conversion) [-> fps] [-> long-test canvas] -> encode
         (create_avpvs_short lib/ffmpeg.py:940, create_avpvs_segment :1003)
  cpvs   decode AVPVS -> fps -> [pad] -> uyvy422 / v210 packing -> encode
         (create_cpvs PC branch lib/ffmpeg.py:1177-1201)
  stall  AVPVS -> stall frames (frozen/black + spinner) or frame freezing
         (bufferer call p03_generateAvPvs.py:236-243, spec PP-STALL-1)
  concat long-test segment AVIs -> one AVI, packets copied (create_avpvs_long_concat :1058, GPU-FFV1 AVIs)
  preview AVPVS decoded here (GPU FFV1) -> ffmpeg's ProRes (create_preview :1250)
  siti   P.910 SI/TI of a SRC (util/SRC_analysis.py hook)

Inputs/outputs ending in .y4m or .raw/.yuv are read/written directly;
anything else goes through ffmpeg pipes.  The device is PIXPATH_DEVICE, else
LOCAL_RANK, else the lowest free GPU slot (pixpath.devslot: the first N
processes of the reference's ParallelRunner pool get N different GPUs).
"""
import argparse
import ast
import hashlib
import json
import os
import sys
from fractions import Fraction

import numpy as np


def _device():
    import torch

    from .devslot import choose_device
    n = torch.cuda.device_count()
    if n == 0:
        raise SystemExit("pixpath: no GPU visible")
    return choose_device(n)


class CountingWriter:
    """Writer wrapper: caps the frame count (-t), remembers the last frame (canvas repeat).
    Forwards device batches (``write_device``) when the inner writer takes them."""

    def __init__(self, inner, frame_bytes, cap=None):
        self.inner, self.fb, self.cap, self.n, self.last = inner, frame_bytes, cap, 0, None
        self.last_dev = None
        if hasattr(inner, "write_device"):
            self.write_device = self._write_device

    def write(self, frames):
        mv = memoryview(frames).cast("B")
        k = len(mv) // self.fb
        if self.cap is not None:
            k = min(k, self.cap - self.n)
        if k <= 0:
            return
        self.inner.write(mv[:k * self.fb])
        self.last = bytes(mv[(k - 1) * self.fb:k * self.fb])
        self.last_dev = None
        self.n += k

    def _write_device(self, frames, stream=None, emit=None):
        import torch
        counts = list(emit) if emit is not None else [1] * frames.n
        if self.cap is not None:
            room = self.cap - self.n
            for i, c in enumerate(counts):
                counts[i] = max(0, min(c, room))
                room -= counts[i]
        total = sum(counts)
        if total <= 0:
            return
        self.inner.write_device(frames, stream, counts)
        self.n += total
        if self.cap is not None:  # keep the last written frame on the device for the canvas repeat
            k = max(i for i, c in enumerate(counts) if c > 0)
            with torch.cuda.stream(stream or torch.cuda.current_stream(frames.device)):
                self.last_dev = frames.storage[k:k + 1].clone()
            self.last = None

    def pad_to_cap(self):
        """overlay eof_action=repeat: the canvas keeps its last frame up to the cap."""
        if self.cap is None or self.n >= self.cap:
            return
        if self.last_dev is not None:
            from .frames import FrameBatch
            fmt = self.inner.fmt
            fb = FrameBatch.interleaved(fmt, self.inner.w, self.inner.h, 1, device=self.last_dev.device,
                                        storage=self.last_dev)
            self.write_device(fb, None, [self.cap - self.n])
        elif self.last is not None:
            while self.n < self.cap:
                self.write(self.last)

    def close(self):
        self.inner.close()


def _open_writer(path, fmt, w, h, rate, vopts, aopts, audio_from, overwrite):
    from . import formats, io as pio
    ext = os.path.splitext(path)[1].lower()
    if ext == ".y4m":
        return pio.Y4MWriter(path, fmt, w, h, rate)
    if ext in (".raw", ".yuv"):
        return pio.RawWriter(path)
    return pio.FFmpegWriter(path, fmt, w, h, rate, vopts, aopts, audio_from=audio_from,
                            overwrite="-y" if overwrite else "-n")  # pragma: no cover


def _skip(path, overwrite):
    if not overwrite and os.path.isfile(path):
        print("pixpath: output %s exists, not overwriting (-y to force)" % path, file=sys.stderr)
        return True
    return False


def _fps_counts(in_rate, out_rate):
    """emit(k): how many output frames show input frame k under vf_fps rounding=near."""
    a, b = Fraction(in_rate), Fraction(out_rate)
    N, D = a.denominator * b.numerator, a.numerator * b.denominator

    def t(i):
        return (2 * i * N + D) // (2 * D)
    return lambda k: t(k + 1) - t(k)


def cmd_avpvs(args):
    import torch
    from . import formats, io as pio, ops
    from .pipeline import Pipeline, Stage
    out = args.output
    if _skip(out, args.y):
        return 0
    dev = _device()
    torch.cuda.set_device(dev)
    if args.ffv1_input:  # an AVPVS written by `--gpu-ffv1` (mobile CPVS scale reads it)
        from .ffv1 import open_avpvs_reader
        rd = open_avpvs_reader(args.input, device=dev)
    else:
        rd = pio.open_reader(args.input)
    W, H = (int(v) for v in args.size.split("x"))
    target = formats.fmt(args.pix_fmt)
    rate = Fraction(args.fps) if args.fps else rd.rate
    if args.overlay_yuv420:
        # create_avpvs_segment: scale into the overlay's yuv420p, then the -pix_fmt
        # conversion -- one chain plan (a single launch, no yuv420p intermediate)
        sc = ops.Scaler(rd.fmt, rd.w, rd.h, target, W, H, flags=args.flags, chain=True)
        stage = Stage(rd.fmt, rd.w, rd.h, target, W, H, lambda s, d, st: sc(s, d, stream=st))
    else:
        sc = ops.Scaler(rd.fmt, rd.w, rd.h, target, W, H, flags=args.flags)
        stage = Stage(rd.fmt, rd.w, rd.h, target, W, H, lambda s, d, st: sc(s, d, stream=st))
    fb = formats.frame_bytes(target, W, H)
    cap = int(round(float(args.duration) * float(rate))) if args.duration else None
    if args.gpu_ffv1:
        # the AVPVS as FFV1 encoded on the GPU, in an AVI written here (video
        # only: the reference's -c:a flac track needs ffmpeg, see _mux_audio)
        from .ffv1 import Ffv1AviWriter
        sl = tuple(int(v) for v in args.ffv1_slices.lower().split("x")) if args.ffv1_slices else None
        inner = Ffv1AviWriter(out, target, W, H, rate, slices=sl, device=dev)
    else:
        inner = _open_writer(out, target, W, H, rate, args.vopts, args.aopts,
                             None if args.aopts.strip() == "-an" else args.input, args.y)
    stall = None
    if args.stall_output and not args.gpu_ffv1:
        # create_avpvs_short of a PVS with stalls: compose the stalled AVPVS
        # (the bufferer step's output) from the frames this pass writes
        stall = _StallOutput(args.stall_output, target, W, H, rate, args.buffer, args.skipping, args.spinner,
                             args.black_frame, args.stall_vopts, args.stall_aopts, args.input, True, dev)
        inner = _Tee(inner, stall.push, fb)
    wr = CountingWriter(inner, fb, cap)
    emit = _fps_counts(rd.rate, rate) if args.fps else None
    Pipeline(stage, batch=args.batch, device=dev).run(rd, wr, emit=emit)
    wr.pad_to_cap()
    rd.close()
    wr.close()
    if args.gpu_ffv1:
        _mux_audio(out, args.input, args.aopts)
    stall_aopts = args.stall_aopts
    if stall is not None:
        stall.close()
        stall_aopts = stall.aopts_written
    elif args.stall_output:
        # the stalled AVPVS from the FFV1 AVPVS just written, at the packet
        # level: pass-through frames are copied packets, only stall frames are
        # composed and encoded (no second decode / encode of the AVPVS)
        from .ffv1 import stall_avi
        events = ast.literal_eval(args.buffer)
        if stall_avi(out, args.stall_output, events, args.skipping, args.spinner, args.black_frame, dev) is None:
            raise SystemExit("pixpath: %s is not a GPU-FFV1 AVI" % out)
        stall_aopts = _mux_stall_audio(args.stall_output, out, args.stall_aopts, events, args.skipping, rate)
    if args.stall_output:
        import json
        with open(_record_path(args.stall_output), "w") as f:
            json.dump(_stall_record(out, args.buffer, args.skipping, args.spinner, args.black_frame, args.pix_fmt,
                                    args.stall_vopts, args.stall_aopts, written_aopts=stall_aopts), f)
    return 0


def _mux_audio(video_avi, audio_src, aopts):
    """Add the source's audio to a video-only AVI with the reference's audio
    options (e.g. `-c:a flac`), stream-copying the GPU-encoded FFV1; without
    ffmpeg (or with -an) the AVI stays video-only."""
    import shutil
    import subprocess
    if aopts.strip() == "-an" or not shutil.which("ffmpeg"):
        if aopts.strip() != "-an":
            print("pixpath: no ffmpeg: %s written without audio" % video_avi, file=sys.stderr)
        return
    tmp = video_avi + ".video.avi"  # pragma: no cover - needs ffmpeg
    os.replace(video_avi, tmp)
    cmd = ["ffmpeg", "-nostdin", "-v", "error", "-y", "-i", tmp, "-i", audio_src, "-map", "0:v", "-map", "1:a?",
           "-c:v", "copy"] + aopts.split() + [video_avi]
    subprocess.run(cmd, check=True)
    os.remove(tmp)


def _mux_stall_audio(video_avi, audio_src, aopts, events, skipping, rate):
    """The stalled AVPVS's audio (bufferer's `-a pcm_s16le`): the source's
    audio with each stall's silence inserted (stall_audio_graph), muxed next to
    the stream-copied FFV1 video.  Returns the audio options actually written:
    `-an` when there is no audio, no ffmpeg, or -an was asked."""
    import shutil
    import subprocess
    from .stall import stall_audio_graph, stall_times
    if aopts.strip() == "-an":
        return "-an"
    if not shutil.which("ffmpeg"):
        print("pixpath: no ffmpeg: %s written without audio" % video_avi, file=sys.stderr)
        return "-an"
    from . import io as pio  # pragma: no cover - needs ffmpeg
    ap = pio.audio_params(audio_src)  # pragma: no cover
    if ap is None:  # pragma: no cover
        return "-an"
    graph = None if skipping else stall_audio_graph(stall_times(events, rate), ap[0], ap[1])  # pragma: no cover
    tmp = video_avi + ".video.avi"  # pragma: no cover
    os.replace(video_avi, tmp)  # pragma: no cover
    cmd = ["ffmpeg", "-nostdin", "-v", "error", "-y", "-i", tmp, "-i", audio_src]  # pragma: no cover
    cmd += (["-filter_complex", graph, "-map", "0:v", "-map", "[aout]"] if graph else
            ["-map", "0:v", "-map", "1:a"])  # pragma: no cover
    subprocess.run(cmd + ["-c:v", "copy"] + aopts.split() + [video_avi], check=True)  # pragma: no cover
    os.remove(tmp)  # pragma: no cover
    return aopts  # pragma: no cover


class _Tee:
    """Writer that also pushes each written frame into a StallStream pusher.
    Frames are pushed as views of the written batch; only the batch's last
    frame -- the one a stall at the start of the next batch shows -- is
    copied, because the caller reuses the batch buffer."""

    def __init__(self, inner, push, frame_bytes):
        self.inner, self.push, self.fb = inner, push, frame_bytes

    def write(self, frames):
        self.inner.write(frames)
        mv = np.frombuffer(memoryview(frames).cast("B"), np.uint8)
        n = len(mv) // self.fb
        for i in range(n):
            f = mv[i * self.fb:(i + 1) * self.fb]
            self.push.push(f.copy() if i == n - 1 else f)

    def close(self):
        self.inner.close()


def cmd_encseg(args):
    """p01 encode_segment's pixel work (lib/ffmpeg.py:794-837): trimmed decode,
    `scale=W:-2:flags=bicubic` (+ the encoder's -pix_fmt conversion) on the
    MI355X, `select` + `fps` as a host frame map; Y4M out (a path or - for
    stdout) for the reference's encoder invocation."""
    import torch
    from . import chain, formats, io as pio, ops
    from .pipeline import Pipeline, Stage
    dev = _device()
    torch.cuda.set_device(dev)
    rd = pio.open_reader(args.input, start=args.start, duration=args.duration)
    W = int(args.width)
    H = chain.scale_height_keep_aspect(rd.w, rd.h, W)
    target = formats.fmt(args.pix_fmt)
    in_rate = Fraction(args.in_fps) if args.in_fps else Fraction(rd.rate)
    out_rate = Fraction(str(args.fps))
    # frames the trimmed decode yields: the -t window at the input rate
    n_in = int(round(Fraction(str(args.duration)) * in_rate)) if args.duration else None
    if n_in is None:
        raise SystemExit("pixpath encseg: --duration is required")
    fmap = chain.select_fps_map(n_in, in_rate, out_rate, args.select or "")
    keep = sorted(set(fmap))
    counts = {k: 0 for k in keep}
    for k in fmap:
        counts[k] += 1
    sel = pio.SelectReader(rd, keep)
    sc = ops.Scaler(rd.fmt, rd.w, rd.h, target, W, H, flags=args.flags)
    stage = Stage(rd.fmt, rd.w, rd.h, target, W, H, lambda s, d, st: sc(s, d, stream=st))
    wr = pio.Y4MWriter(args.output, target, W, H, out_rate)
    Pipeline(stage, batch=args.batch, device=dev).run(sel, wr, emit=lambda i: counts[keep[i]])
    sel.close()
    wr.close()
    return 0


def cmd_cpvs(args):
    import torch
    from . import formats, io as pio, ops
    from .frames import FrameBatch
    from .pipeline import Pipeline, Stage
    out = args.output
    if _skip(out, args.y):
        return 0
    dev = _device()
    torch.cuda.set_device(dev)
    if args.gpu_ffv1:  # an FFV1 AVPVS written by `avpvs --gpu-ffv1`: decoded on the GPU
        from .ffv1 import open_avpvs_reader
        rd = open_avpvs_reader(args.input, device=dev)
    else:
        rd = pio.open_reader(args.input)
    W, H = (rd.w, rd.h) if not args.pad else (int(v) for v in args.pad.split("x"))
    W, H = int(W), int(H)
    cur_fmt = rd.fmt
    steps = []
    fused = (args.vcodec == "rawvideo" and args.pix_fmt == "uyvy422" and cur_fmt.depth == 8) or \
            (args.vcodec == "v210" and cur_fmt.depth == 10)
    if fused:  # one pass: pad + chroma conversion + packing (pp_cpvs_execute)
        steps.append(("cpvs",))
    elif args.pad:
        steps.append(("pad", W, H))
    if fused:
        out_fmt = formats.fmt("uyvy422" if cur_fmt.depth == 8 else "v210")
    elif args.vcodec == "rawvideo" and args.pix_fmt == "uyvy422":
        out_fmt = formats.fmt("uyvy422")
        steps.append(("scale", ops.Scaler(cur_fmt, W, H, "uyvy422", W, H, flags="bicubic")))
    elif args.vcodec == "v210":
        out_fmt = formats.fmt("v210")
        if cur_fmt.name != "yuv422p10le":
            steps.append(("scale", ops.Scaler(cur_fmt, W, H, "yuv422p10le", W, H, flags="bicubic")))
        steps.append(("v210",))
    else:  # -a/--rawvideo: keep the AVPVS format
        out_fmt = cur_fmt
    cache = {}

    def tmp(key, f, n, dev_):
        t = cache.get((key, n))
        if t is None:
            t = cache[(key, n)] = FrameBatch(f, W, H, n, device=dev_)
        return t

    def process(src, dst, stream):
        cur = src
        for i, st in enumerate(steps):
            last = i == len(steps) - 1
            if st[0] == "cpvs":
                nxt = dst
                ops.cpvs(cur, W, H, out_fmt, dst=nxt, stream=stream)
            elif st[0] == "pad":
                nxt = dst if last else tmp("pad", cur.fmt, cur.n, cur.device)
                ops.pad(cur, W, H, dst=nxt, stream=stream)
            elif st[0] == "scale":
                nxt = dst if last else tmp("scale", st[1].dst_fmt, cur.n, cur.device)
                st[1](cur, nxt, stream=stream)
            else:
                nxt = dst
                ops.v210_pack(cur, dst=nxt, stream=stream)
            cur = nxt
        if not steps:
            for p in range(len(dst.planes)):
                dst.view(p).copy_(src.view(p))
    stage = Stage(rd.fmt, rd.w, rd.h, out_fmt, W, H, process)
    inner = _open_writer(out, out_fmt, W, H, Fraction(args.fps), "-c:v %s" % args.vcodec + (
        "" if args.vcodec == "v210" else " -pix_fmt %s" % args.pix_fmt), args.aopts, args.input, args.y)
    emit = _fps_counts(rd.rate, Fraction(args.fps))
    Pipeline(stage, batch=args.batch, device=dev).run(rd, inner, emit=emit)
    rd.close()
    inner.close()
    return 0


from .stall import stall_schedule  # noqa: E402,F401  (PP-STALL-1, re-exported for callers/tests)


class _StallOutput:
    """The PP-STALL-1 output side (p03_generateAvPvs.py:236-243): a writer
    plus a frame-by-frame StallStream pusher.  Input frames pass through;
    stall runs are composed on the GPU from the retained frame (frozen frame or
    black + spinner) and the audio gets the stalls' silence.  Shared by
    `cli stall` (reading the AVPVS) and `cli avpvs --stall-output` (fed by
    the AVPVS writer itself, no second decode)."""

    def __init__(self, out, fmt, w, h, rate, buffer, skipping, spinner_path, black_frame, vopts, aopts,
                 audio_input, overwrite, dev, gpu_ffv1=False):
        """gpu_ffv1: the output is an FFV1 AVI coded on the GPU (a decoded
        input that is not a GPU-FFV1 AVI); its audio is muxed by close()."""
        import torch
        from . import io as pio, ops, spinner
        from .frames import FrameBatch
        from .stall import StallStream, stall_audio_graph, stall_times
        device = torch.device("cuda", dev)
        events = ast.literal_eval(buffer)
        delays = None
        if not skipping:
            anim, delays = spinner.load_apng(spinner_path)
            ops.spinner_upload(anim, fmt, device=dev)
        audio_from, graph = None, None
        self.out, self.gpu_ffv1, self.events, self.skipping, self.rate = out, gpu_ffv1, events, skipping, rate
        self.audio_input, self.aopts = audio_input, aopts
        self.aopts_written = "-an"
        if not gpu_ffv1 and aopts.strip() != "-an" and \
                os.path.splitext(out)[1].lower() not in (".y4m", ".raw", ".yuv"):
            ap = pio.audio_params(audio_input)  # pragma: no cover - needs ffprobe
            if ap is not None:
                audio_from = audio_input
                if not skipping:
                    graph = stall_audio_graph(stall_times(events, rate), ap[0], ap[1])
        if gpu_ffv1:  # FFV1 encoded on the GPU into an AVI; audio muxed on close
            from .ffv1 import Ffv1AviWriter
            self.wr = Ffv1AviWriter(out, fmt, w, h, rate, device=dev)
        elif audio_from:  # pragma: no cover - needs ffmpeg
            self.aopts_written = aopts
            self.wr = pio.FFmpegWriter(out, fmt, w, h, rate, vopts, aopts, audio_from=audio_from,
                                       overwrite="-y" if overwrite else "-n", audio_filter=graph)
        else:
            self.wr = _open_writer(out, fmt, w, h, rate, vopts, aopts, None, overwrite)
        self.fb = fb = formats_frame_bytes(fmt, w, h)
        self.fmt, self.w, self.h, self.device = fmt, w, h, device
        self.src_b = FrameBatch.interleaved(fmt, w, h, 1, device=device)
        self.blk = 256
        self.dst_b = FrameBatch.interleaved(fmt, w, h, self.blk, device=device)
        self.host = torch.empty((self.blk, fb), dtype=torch.uint8).pin_memory()
        self.push = StallStream(events, rate, skipping, delays, black_frame=black_frame).pusher(
            self.wr.write, self._emit_stall)

    def _emit_stall(self, f, spin):
        import torch
        from . import ops
        from .frames import FrameBatch
        fmt, w, h, fb, device = self.fmt, self.w, self.h, self.fb, self.device
        if f is not None:
            self.src_b.storage.copy_(torch.from_numpy(np.asarray(f)).view(1, fb).to(device, non_blocking=False))
        for i in range(0, len(spin), self.blk):
            part = spin[i:i + self.blk]
            n = len(part)
            ops.stall_compose(self.src_b, [0 if f is not None else -1] * n, part,
                              dst=FrameBatch.interleaved(fmt, w, h, n, device=device,
                                                         storage=self.dst_b.storage[:n]))
            self.host[:n].copy_(self.dst_b.storage[:n])  # synchronous D2H into pinned memory
            self.wr.write(self.host[:n].numpy())

    def close(self):
        n = self.push.close()
        self.wr.close()
        if self.gpu_ffv1:
            self.aopts_written = _mux_stall_audio(self.out, self.audio_input, self.aopts, self.events, self.skipping,
                                                  self.rate)
        return n


def formats_frame_bytes(fmt, w, h):
    from . import formats
    return formats.frame_bytes(fmt, w, h)


# Provenance of a stalled AVPVS written by `cli avpvs --stall-output`: the
# bufferer step (`cli stall`) keeps that output when this record matches its
# own arguments and the AVPVS it would read is the one the record names.
def _stall_record(input_path, buffer, skipping, spinner_path, black_frame, pix_fmt, vopts, aopts, written_aopts=None):
    st = os.stat(input_path)
    spin = None
    if not skipping:
        with open(spinner_path, "rb") as f:
            spin = hashlib.sha256(f.read()).hexdigest()
    return {"input": os.path.abspath(input_path), "input_size": st.st_size, "input_mtime_ns": st.st_mtime_ns,
            "buffer": buffer, "skipping": bool(skipping), "spinner_sha256": spin, "black_frame": bool(black_frame),
            "pix_fmt": pix_fmt, "vopts": vopts, "aopts": aopts,
            "aopts_written": aopts if written_aopts is None else written_aopts}


def _record_path(out):
    return out + ".pixpath-stall.json"


def cmd_stall(args):
    """bufferer replacement (p03_generateAvPvs.py:236-243, spec PP-STALL-1):
    the AVPVS is read once, in order; input frames pass through untouched,
    stall runs are composed on the GPU from the one retained frame (frozen
    frame or black + spinner), and the audio gets the stalls' silence.
    An output the AVPVS pass already composed (`cli avpvs --stall-output`,
    same arguments, same AVPVS) is kept as is: no second decode/encode."""
    import json
    import torch
    from . import io as pio
    out = args.output
    rec = _record_path(out)
    if os.path.isfile(rec) and os.path.isfile(out):
        try:
            want = _stall_record(args.input, args.buffer, args.skipping, args.spinner, args.black_frame,
                                 args.pix_fmt, args.vopts, args.aopts)
            have = json.load(open(rec))
            want["aopts_written"] = have.get("aopts_written")  # what the fused pass could write
        except (OSError, ValueError):
            want, have = None, {}
        if want == have:
            print("pixpath: %s was composed with the AVPVS pass; kept" % out, file=sys.stderr)
            return 0
        os.remove(out)  # a speculative output for other arguments: ours to replace
        os.remove(rec)
    elif _skip(out, args.y):
        return 0
    dev = _device()
    torch.cuda.set_device(dev)
    gpu_out = getattr(args, "gpu_ffv1_out", args.gpu_ffv1)
    if args.gpu_ffv1 and gpu_out:
        from .ffv1 import open_avpvs_reader, stall_avi
        events = ast.literal_eval(args.buffer)
        n = stall_avi(args.input, out, events, args.skipping, args.spinner, args.black_frame, dev)
        if n is not None:  # packet level: copied input packets + encoded stall frames
            from .avi import scan
            _mux_stall_audio(out, args.input, args.aopts, events, args.skipping, scan(args.input)[0]["rate"])
            return 0
        rd = open_avpvs_reader(args.input, device=dev)  # not pixpath's FFV1: decode it (GPU or ffmpeg)
    elif args.gpu_ffv1:
        from .ffv1 import open_avpvs_reader
        rd = open_avpvs_reader(args.input, device=dev)
    else:
        rd = pio.open_reader(args.input)
    so = _StallOutput(out, rd.fmt, rd.w, rd.h, rd.rate, args.buffer, args.skipping, args.spinner, args.black_frame,
                      args.vopts, args.aopts, args.input, args.y, dev, gpu_ffv1=gpu_out)
    B = max(1, int(args.batch))
    # the input in batches, two buffers in turn: the pusher references the
    # frame before a stall, which must survive the next batch's read
    bufs = [np.empty((B, rd.frame_bytes), np.uint8) for _ in range(2)]
    j = 0
    while True:
        buf = bufs[j & 1]
        k = rd.read_into(buf, B)
        for i in range(k):
            so.push.push(buf[i])
        j += 1
        if k < B:
            break
    rd.close()
    so.close()
    return 0


def cmd_concat(args):
    """create_avpvs_long_concat (lib/ffmpeg.py:1058-1105: `ffmpeg -f concat
    -safe 0 -i <filelist> -c:v copy -t <total>`) for FFV1 AVIs of one
    configuration record: the segment canvases' packets copied in filelist
    order, each with its keyframe flag (an FFmpeg-made GOP stream's inter
    frames are not marked key in the index), cut after round(total * rate)
    frames.  No pixels are decoded."""
    from . import avi
    from .ffv1 import packet_is_keyframe
    out = args.output
    if _skip(out, args.y):
        return 0
    files = []
    with open(args.filelist) as fh:
        for line in fh:
            line = line.strip()
            if line.startswith("file "):
                files.append(line[5:].strip().strip("'"))
    if not files:
        raise SystemExit("pixpath concat: %s lists no files" % args.filelist)
    scans = [avi.scan(f) for f in files]
    i0 = scans[0][0]
    for f, (info, _) in zip(files, scans):
        if info.get("fourcc") != b"FFV1" or info.get("extradata") != i0.get("extradata") or \
                (info["w"], info["h"], info["rate"]) != (i0["w"], i0["h"], i0["rate"]):
            raise SystemExit("pixpath concat: %s is not a GPU-FFV1 AVI matching %s" % (f, files[0]))
    cap = int(round(Fraction(str(args.duration)) * i0["rate"])) if args.duration else None
    wr = avi.AviWriter(out, i0["w"], i0["h"], i0["rate"], extradata=i0["extradata"], info=i0.get("tags"))
    n = 0
    try:
        for f, (_, index) in zip(files, scans):
            with open(f, "rb") as fh:
                for off, size in index:
                    if cap is not None and n >= cap:
                        break
                    fh.seek(off)
                    pkt = fh.read(size)
                    wr.write_packet(pkt, key=packet_is_keyframe(pkt))
                    n += 1
    except BaseException:
        wr.abort()
        raise
    wr.close()
    return 0


def cmd_preview(args):
    """create_preview (lib/ffmpeg.py:1250-1259: `ffmpeg -i <avpvs> -c:v prores
    -c:a aac <preview>`) with the AVPVS decoded here -- on the GPU when it is
    pixpath's FFV1 -- and piped to ffmpeg's ProRes encoder with the AVPVS's
    audio; no pixel work besides the decode."""
    import torch
    out = args.output
    if _skip(out, args.y):
        return 0
    dev = _device()
    torch.cuda.set_device(dev)
    from .ffv1 import open_avpvs_reader
    rd = open_avpvs_reader(args.input, device=dev)
    wr = _open_writer(out, rd.fmt, rd.w, rd.h, rd.rate, args.vopts, args.aopts, args.input, args.y)
    B = max(1, int(args.batch))
    buf = np.empty((B, rd.frame_bytes), np.uint8)
    while True:
        k = rd.read_into(buf, B)
        if k:
            wr.write(buf[:k])
        if k < B:
            break
    rd.close()
    wr.close()
    return 0


def _black(fmt, w, h):
    from . import formats, io as pio
    planes = [np.full((1, r, c), (16 if p == 0 else 128) << (fmt.depth - 8),
                      np.uint16 if fmt.bytes_per_sample == 2 else np.uint8)
              for p, (r, c) in enumerate(formats.plane_shapes(fmt, w, h))]
    return pio.join_planes(planes)


def cmd_siti(args):
    from . import siti
    si, ti = siti.siti_of_file(args.input, batch=args.batch, normalize=args.normalize)
    SI, TI = siti.siti_summary(si, ti)
    res = {"file": os.path.basename(args.input), "si": SI, "ti": TI, "frames": int(len(si))}
    if args.per_frame:
        res["si_frames"] = [float(v) for v in si]
        res["ti_frames"] = [None if np.isnan(v) else float(v) for v in ti]
    print(json.dumps(res))
    return 0


def _avi(path):
    return str(path).lower().endswith(".avi")


def main(argv=None):
    ap = argparse.ArgumentParser(prog="pixpath.cli")
    sub = ap.add_subparsers(dest="cmd", required=True)

    def common(p):
        g = p.add_mutually_exclusive_group()
        g.add_argument("-y", action="store_true", help="overwrite output")
        g.add_argument("-n", action="store_true", help="never overwrite (default)")
        p.add_argument("--input", required=True)
        p.add_argument("--batch", type=int, default=32)
        p.add_argument("--vopts", default="-c:v ffv1")
        p.add_argument("--aopts", default="-an")
        p.add_argument("output")

    p = sub.add_parser("avpvs")
    common(p)
    p.add_argument("--size", required=True)
    p.add_argument("--flags", default="bicubic")
    p.add_argument("--pix-fmt", required=True)
    p.add_argument("--fps", default=None)
    p.add_argument("--duration", default=None)
    p.add_argument("--overlay-yuv420", action="store_true")
    # the stalled AVPVS in the same pass (p03's bufferer step, fused)
    p.add_argument("--stall-output", default=None)
    p.add_argument("--buffer", default="[]")
    p.add_argument("--spinner", default=None)
    p.add_argument("--skipping", action="store_true")
    p.add_argument("--black-frame", action="store_true")
    p.add_argument("--stall-vopts", default="-c:v ffv1")
    p.add_argument("--stall-aopts", default="-c:a pcm_s16le")
    p.add_argument("--gpu-ffv1", action="store_true", help="FFV1 encoded on the GPU into an AVI (pixpath.avi)")
    p.add_argument("--ffv1-slices", default=None, help="slice grid HxV of the GPU FFV1 (default PIXPATH_FFV1_SLICES, 8x8)")
    p.add_argument("--ffv1-input", action="store_true", help="input is a --gpu-ffv1 AVI: decode it on the GPU")
    p.set_defaults(fn=cmd_avpvs)

    p = sub.add_parser("encseg")
    p.add_argument("--input", required=True)
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--start", default=None)
    p.add_argument("--duration", default=None)
    p.add_argument("--width", required=True)
    p.add_argument("--flags", default="bicubic")
    p.add_argument("--pix-fmt", required=True)
    p.add_argument("--select", default="")
    p.add_argument("--fps", required=True)
    p.add_argument("--in-fps", default=None)
    p.add_argument("output")
    p.set_defaults(fn=cmd_encseg)

    p = sub.add_parser("cpvs")
    common(p)
    p.add_argument("--fps", default="60")
    p.add_argument("--vcodec", required=True)
    p.add_argument("--pix-fmt", required=True)
    p.add_argument("--pad", default=None)
    p.add_argument("--gpu-ffv1", action="store_true", help="input is an FFV1 AVI: decode it on the GPU")
    p.set_defaults(fn=cmd_cpvs)

    p = sub.add_parser("stall")
    common(p)
    p.add_argument("--buffer", required=True)
    p.add_argument("--pix-fmt", default=None)
    p.add_argument("--spinner", default=None)
    p.add_argument("--skipping", action="store_true")
    p.add_argument("--black-frame", action="store_true")
    p.add_argument("--gpu-ffv1", action="store_true", help="FFV1 AVI in and out, coded on the GPU")
    p.set_defaults(fn=cmd_stall)

    p = sub.add_parser("concat")
    g = p.add_mutually_exclusive_group()
    g.add_argument("-y", action="store_true", help="overwrite output")
    g.add_argument("-n", action="store_true", help="never overwrite (default)")
    p.add_argument("--filelist", required=True)
    p.add_argument("--duration", default=None)
    p.add_argument("output")
    p.set_defaults(fn=cmd_concat)

    p = sub.add_parser("preview")
    common(p)
    p.set_defaults(fn=cmd_preview)

    p = sub.add_parser("siti")
    p.add_argument("--input", required=True)
    p.add_argument("--batch", type=int, default=120)
    p.add_argument("--per-frame", action="store_true")
    p.add_argument("--normalize", action="store_true", help="SI/TI on the 8-bit scale (/ 2^(bitdepth-8))")
    p.set_defaults(fn=cmd_siti)

    args = ap.parse_args(argv)
    # GPU FFV1 applies to AVI files (the reference's AVPVS container); Y4M /
    # raw files and other containers keep their own readers and writers
    if getattr(args, "ffv1_input", False):
        args.ffv1_input = _avi(args.input)
    if getattr(args, "gpu_ffv1", False):
        if args.cmd == "avpvs":
            args.gpu_ffv1 = _avi(args.output)
        elif args.cmd == "cpvs":
            args.gpu_ffv1 = _avi(args.input)
        elif args.cmd == "stall":
            args.gpu_ffv1 = _avi(args.input)
            args.gpu_ffv1_out = _avi(args.output)
    return args.fn(args)


if __name__ == "__main__":
    sys.exit(main())
