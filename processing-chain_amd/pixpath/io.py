"""Raw-frame I/O for the host pipeline: Y4M / raw files, and ffmpeg/ffprobe pipes.

ffmpeg stays the bitstream decoder/encoder (as in the reference); between the
decode pipe and the encode pipe frames are dense raw planes (Y|U|V per frame),
which is also the layout of the pinned host buffers and of the frame-
interleaved device batches (pixpath.frames.FrameBatch.interleaved).
"""
import json
import os
import shlex
import subprocess
from fractions import Fraction

import numpy as np

from . import formats

Y4M_TAGS = {
    "420jpeg": "yuv420p", "420paldv": "yuv420p", "420mpeg2": "yuv420p", "420": "yuv420p",
    "422": "yuv422p", "444": "yuv444p", "420p10": "yuv420p10le", "422p10": "yuv422p10le", "444p10": "yuv444p10le",
}
Y4M_OUT = {"yuv420p": "420mpeg2", "yuv422p": "422", "yuv444p": "444", "yuv420p10le": "420p10",
           "yuv422p10le": "422p10", "yuv444p10le": "444p10"}


class Reader:
    fmt = None
    w = h = 0
    rate = Fraction(60)

    @property
    def frame_bytes(self):
        return formats.frame_bytes(self.fmt, self.w, self.h)

    def read_into(self, buf, n):
        """Fill up to n dense frames into a writable bytes-like `buf`; return frames read."""
        fb = self.frame_bytes
        mv = memoryview(buf).cast("B")
        got = 0
        while got < n:
            if not self._read_frame(mv[got * fb:(got + 1) * fb]):
                break
            got += 1
        return got

    def batches(self, n):
        """Yield lists of [k, rows, cols] numpy planes, k <= n (tests / analysis)."""
        fb = self.frame_bytes
        buf = bytearray(fb * n)
        while True:
            k = self.read_into(buf, n)
            if k == 0:
                return
            yield split_planes(np.frombuffer(bytes(buf[:k * fb]), np.uint8).reshape(k, fb), self.fmt, self.w, self.h)
            if k < n:
                return

    def close(self):
        pass


def split_planes(frames_u8, f, w, h):
    """[k, frame_bytes] uint8 -> list of [k, rows, cols] planes (views)."""
    f = formats.fmt(f)
    out, off = [], 0
    dt = np.uint16 if f.bytes_per_sample == 2 and not f.packed else np.uint8
    for r, c in formats.plane_shapes(f, w, h):
        nb = r * c * (1 if f.packed else f.bytes_per_sample)
        out.append(frames_u8[:, off:off + nb].view(dt).reshape(-1, r, c))
        off += nb
    return out


def join_planes(planes):
    """list of [k, rows, cols] planes -> [k, frame_bytes] uint8."""
    k = planes[0].shape[0]
    return np.concatenate([np.ascontiguousarray(p).view(np.uint8).reshape(k, -1) for p in planes], axis=1)


def _readexact(fh, mv):
    n = 0
    while n < len(mv):
        k = fh.readinto(mv[n:])
        if not k:
            return n
        n += k
    return n


class Y4MReader(Reader):
    def __init__(self, path_or_fh):
        self.fh = open(path_or_fh, "rb") if isinstance(path_or_fh, str) else path_or_fh
        hdr = self.fh.readline().decode().split()
        if hdr[0] != "YUV4MPEG2":
            raise ValueError("not a YUV4MPEG2 stream")
        tags = {t[0]: t[1:] for t in hdr[1:]}
        self.w, self.h = int(tags["W"]), int(tags["H"])
        if "F" in tags:
            a, b = tags["F"].split(":")
            self.rate = Fraction(int(a), int(b))
        self.fmt = formats.fmt(Y4M_TAGS[tags.get("C", "420jpeg")])

    def _read_frame(self, mv):
        line = self.fh.readline()
        if not line:
            return False
        if not line.startswith(b"FRAME"):
            raise ValueError("bad Y4M frame header")
        return _readexact(self.fh, mv) == len(mv)

    def close(self):
        self.fh.close()


class RawReader(Reader):
    def __init__(self, path_or_fh, f, w, h, rate=60):
        self.fh = open(path_or_fh, "rb") if isinstance(path_or_fh, str) else path_or_fh
        self.fmt, self.w, self.h, self.rate = formats.fmt(f), int(w), int(h), Fraction(rate)

    def _read_frame(self, mv):
        return _readexact(self.fh, mv) == len(mv)

    def close(self):
        self.fh.close()


class FFmpegReader(RawReader):  # pragma: no cover - needs ffmpeg
    """Decode any container through `ffmpeg ... -f rawvideo -pix_fmt F pipe:1`
    (optionally trimmed like the reference's p01 encode: `-ss S -i IN -t D`)."""

    def __init__(self, path, f=None, w=None, h=None, rate=None, start=None, duration=None):
        st = probe(path)["stream"]
        f = f or st["pix_fmt"]
        pre = ["-ss", str(start)] if start is not None else []
        post = ["-t", str(duration)] if duration is not None else []
        self.proc = subprocess.Popen(["ffmpeg", "-nostdin", "-v", "error"] + pre + ["-i", path] + post +
                                     ["-f", "rawvideo", "-pix_fmt", f, "pipe:1"], stdout=subprocess.PIPE,
                                     bufsize=1 << 24)
        super().__init__(self.proc.stdout, f, w or st["width"], h or st["height"],
                         rate or Fraction(st["r_frame_rate"]))

    def close(self):
        self.proc.stdout.close()
        if self.proc.wait():
            raise RuntimeError("ffmpeg decode failed")


class Writer:
    def write(self, frames_u8):
        """frames_u8: [k, frame_bytes] uint8 (or bytes-like of k dense frames)."""
        raise NotImplementedError

    def close(self):
        pass


class Y4MWriter(Writer):
    def __init__(self, path, f, w, h, rate=60):
        import sys
        self.fh = sys.stdout.buffer if path == "-" else open(path, "wb")
        r = Fraction(rate)
        self.fb = formats.frame_bytes(f, w, h)
        self.fh.write(("YUV4MPEG2 W%d H%d F%d:%d Ip A1:1 C%s\n" % (w, h, r.numerator, r.denominator,
                                                                  Y4M_OUT[formats.fmt(f).name])).encode())

    def write(self, frames_u8):
        mv = memoryview(frames_u8).cast("B")
        for i in range(len(mv) // self.fb):
            self.fh.write(b"FRAME\n")
            self.fh.write(mv[i * self.fb:(i + 1) * self.fb])

    def close(self):
        self.fh.close()


class RawWriter(Writer):
    def __init__(self, path):
        self.fh = open(path, "wb")

    def write(self, frames_u8):
        self.fh.write(memoryview(frames_u8).cast("B"))

    def close(self):
        self.fh.close()


class FFmpegWriter(Writer):  # pragma: no cover - needs ffmpeg
    """Encode raw frames with the reference's encoder options (e.g. FFV1 / v210 / rawvideo)."""

    def __init__(self, path, f, w, h, rate, vopts, aopts="-an", audio_from=None, overwrite="-y", extra_in="",
                 audio_filter=None, sar="1/1"):
        r = Fraction(rate)
        cmd = "ffmpeg -nostdin -v error {ow} -f rawvideo -pix_fmt {pf} -s {w}x{h} -r {num}/{den} -i pipe:0 ".format(
            ow=overwrite, pf=formats.fmt(f).name if not formats.fmt(f).packed else
            ("uyvy422" if formats.fmt(f).id == formats.UYVY422 else "yuv422p10le"),
            w=w, h=h, num=r.numerator, den=r.denominator)
        if audio_from and audio_filter:
            cmd += "-i {} -filter_complex {} -map 0:v -map '[aout]' ".format(shlex.quote(audio_from),
                                                                          shlex.quote(audio_filter))
        elif audio_from:
            cmd += "-i {} -map 0:v -map 1:a? ".format(shlex.quote(audio_from))
        # a raw pipe carries no sample aspect ratio: restate the 1:1 the reference's
        # chains set (setsar=1/1, lib/ffmpeg.py:992, :1038, :1213) or inherit
        sar_opt = "-filter:v setsar={}".format(sar) if sar else ""
        cmd += "{} {} {} {} {}".format(extra_in, sar_opt, vopts, aopts, shlex.quote(path))
        self.proc = subprocess.Popen(cmd, shell=True, stdin=subprocess.PIPE, bufsize=1 << 24)

    def write(self, frames_u8):
        self.proc.stdin.write(memoryview(frames_u8).cast("B"))

    def close(self):
        self.proc.stdin.close()
        if self.proc.wait():
            raise RuntimeError("ffmpeg encode failed")


class TrimmedReader(Reader):
    """Frames [skip, skip + count) of another reader (input seeking -ss / -t on
    files read directly; exact when the times are whole frame periods)."""

    def __init__(self, inner, skip, count=None):
        self.inner, self.left = inner, count
        self.fmt, self.w, self.h, self.rate = inner.fmt, inner.w, inner.h, inner.rate
        if skip:
            buf = bytearray(inner.frame_bytes)
            for _ in range(skip):
                if not inner._read_frame(memoryview(buf)):
                    break

    def _read_frame(self, mv):
        if self.left is not None:
            if self.left <= 0:
                return False
            self.left -= 1
        return self.inner._read_frame(mv)

    def close(self):
        self.inner.close()


class SelectReader(Reader):
    """Only the input frames whose index is in `keep` (a sorted list): frames a
    select/fps map drops are never sent to the GPU."""

    def __init__(self, inner, keep):
        self.inner, self.keep, self.i, self.k = inner, keep, 0, 0
        self.fmt, self.w, self.h, self.rate = inner.fmt, inner.w, inner.h, inner.rate
        self._skip = bytearray(inner.frame_bytes)

    def _read_frame(self, mv):
        if self.k >= len(self.keep):
            return False
        while self.i < self.keep[self.k]:
            if not self.inner._read_frame(memoryview(self._skip)):
                return False
            self.i += 1
        ok = self.inner._read_frame(mv)
        self.i += 1
        self.k += 1
        return ok

    def close(self):
        self.inner.close()


class LumaReader:
    """The luma plane of every frame, nothing else (P.910 SI/TI reads luma
    only): Y4M / raw files seek past the chroma planes; any other container
    is decoded by ffmpeg straight to `-pix_fmt gray` / `gray10le`, so the
    decode pipe, the pinned buffers and PCIe carry 1/2 (4:2:2) or 2/3 (4:2:0)
    fewer bytes than full frames.  read_into(buf, n) fills n dense
    [h * w * bytes_per_sample] luma frames."""

    def __init__(self, path, f=None, w=None, h=None, rate=None):
        """path: a file name, or an open binary Y4M stream (e.g. a pipe)."""
        ext = os.path.splitext(path)[1].lower() if isinstance(path, str) else ".y4m"
        self.proc = None
        self.skip = 0
        if ext == ".y4m":
            y = Y4MReader(path)
            self.fh, fmt, self.w, self.h, self.rate = y.fh, y.fmt, y.w, y.h, y.rate
            self.y4m = True
        elif ext in (".raw", ".yuv"):
            fmt = formats.fmt(f)
            self.fh, self.w, self.h, self.rate = open(path, "rb"), int(w), int(h), Fraction(rate or 60)
            self.y4m = False
        else:  # pragma: no cover - needs ffmpeg
            st = probe(path)["stream"]
            fmt = formats.fmt(f or st["pix_fmt"]) if (f or st["pix_fmt"]) in formats.NAMES else None
            depth = fmt.depth if fmt else (10 if "10" in st["pix_fmt"] else 8)
            self.w, self.h = int(w or st["width"]), int(h or st["height"])
            self.rate = Fraction(rate or st["r_frame_rate"])
            self.proc = subprocess.Popen(["ffmpeg", "-nostdin", "-v", "error", "-i", path, "-f", "rawvideo",
                                          "-pix_fmt", "gray10le" if depth > 8 else "gray", "pipe:1"],
                                         stdout=subprocess.PIPE, bufsize=1 << 24)
            self.fh, self.y4m, self.depth = self.proc.stdout, False, depth
        if self.proc is None:
            self.depth = fmt.depth
            self.skip = formats.frame_bytes(fmt, self.w, self.h) - self.luma_bytes
        try:
            self.seekable = self.fh.seekable()
        except (AttributeError, OSError):
            self.seekable = False
        self._scratch = None if self.seekable else bytearray(self.skip)

    @property
    def luma_bytes(self):
        return self.w * self.h * (2 if self.depth > 8 else 1)

    def read_into(self, buf, n):
        lb = self.luma_bytes
        mv = memoryview(buf).cast("B")
        got = 0
        while got < n:
            if self.y4m:
                line = self.fh.readline()
                if not line:
                    break
                if not line.startswith(b"FRAME"):
                    raise ValueError("bad Y4M frame header")
            if _readexact(self.fh, mv[got * lb:(got + 1) * lb]) != lb:
                break
            if self.skip:
                if self.seekable:
                    self.fh.seek(self.skip, os.SEEK_CUR)
                else:
                    _readexact(self.fh, memoryview(self._scratch))
            got += 1
        return got

    def close(self):
        self.fh.close()
        if self.proc is not None and self.proc.wait():  # pragma: no cover - needs ffmpeg
            raise RuntimeError("ffmpeg decode failed")


def open_reader(path, f=None, w=None, h=None, rate=None, start=None, duration=None):
    """Reader for a Y4M / raw file (read directly) or any container (ffmpeg
    decode pipe); start/duration trim like `-ss start -i path -t duration`."""
    ext = os.path.splitext(path)[1].lower()
    if ext in (".y4m", ".raw", ".yuv"):
        rd = Y4MReader(path) if ext == ".y4m" else RawReader(path, f, w, h, rate or 60)
        if start is None and duration is None:
            return rd
        r = Fraction(rd.rate)
        skip = int(round(Fraction(str(start or 0)) * r))
        count = None if duration is None else int(round(Fraction(str(duration)) * r))
        return TrimmedReader(rd, skip, count)
    return FFmpegReader(path, f, w, h, rate, start=start, duration=duration)


def audio_params(path):  # pragma: no cover - needs ffprobe
    """(sample_rate, channel_layout) of the first audio stream, or None."""
    try:
        out = subprocess.run(["ffprobe", "-loglevel", "error", "-select_streams", "a", "-show_streams", "-of",
                              "json", path], check=True, capture_output=True).stdout
    except (OSError, subprocess.CalledProcessError):
        return None
    st = json.loads(out).get("streams", [])
    if not st:
        return None
    return int(st[0]["sample_rate"]), st[0].get("channel_layout") or "stereo"


def probe(path):
    """Decode-side stream description for the readers: Y4M headers are parsed,
    anything else is asked of ffprobe (raw r_frame_rate, e.g. "60000/1001").
    The reference's metadata calls (get_src_info / get_stream_size /
    get_segment_info, with their normalisations) are pixpath.probe."""
    if path.lower().endswith(".y4m"):
        r = Y4MReader(path)
        st = {"width": r.w, "height": r.h, "coded_width": r.w, "coded_height": r.h, "pix_fmt": r.fmt.name,
              "r_frame_rate": str(r.rate.numerator // r.rate.denominator) if r.rate.denominator == 1 else
              "%d/%d" % (r.rate.numerator, r.rate.denominator), "codec_name": "rawvideo"}
        r.close()
        return {"stream": st, "sizes": {"v": os.path.getsize(path), "a": 0}}
    out = subprocess.run(["ffprobe", "-loglevel", "error", "-select_streams", "v", "-show_streams", "-of", "json",
                          path], check=True, capture_output=True).stdout  # pragma: no cover
    st = json.loads(out)["streams"][0]  # pragma: no cover
    sizes = {}
    for sw in ("v", "a"):  # pragma: no cover
        o = subprocess.run(["ffprobe", "-loglevel", "error", "-select_streams", sw, "-show_entries", "packet=size",
                            "-of", "compact=p=0:nk=1", path], check=True, capture_output=True).stdout.decode()
        sizes[sw] = sum(int(x) for x in o.split("\n") if x)
    return {"stream": st, "sizes": sizes}  # pragma: no cover
