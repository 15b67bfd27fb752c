"""AVI (with the OpenDML 2.0 extension) for one video stream of compressed
frame packets -- the container of the reference's AVPVS (`<pvs>.avi`,
lib/ffmpeg.py:951-954, FFV1 video) when the FFV1 encode runs on the GPU.

Layout written (RIFF chunks, little-endian):
  RIFF 'AVI ' [ LIST 'hdrl' [ avih, LIST 'strl' [ strh, strf (BITMAPINFOHEADER
  + codec private data), indx (OpenDML super index) ], LIST 'odml' [ dmlh ] ],
  [ LIST 'INFO' [ ISFT ... ] ], LIST 'movi' [ '00dc' packets..., ix00 (standard
  index) ], idx1 ]
  RIFF 'AVIX' [ LIST 'movi' [ '00dc'..., ix00 ] ] ...   (every RIFF < 1 GiB)
The reader walks the chunks (it needs no index).  Round trips are tested
here; acceptance by FFmpeg's avidec is unpinned (no FFmpeg in this
environment).
"""
import os
import struct
from fractions import Fraction

RIFF_LIMIT = 1 << 30  # bytes per RIFF (OpenDML readers expect < 1 GiB before AVIX)
SUPER_ENTRIES = 256   # indx slots reserved (one per RIFF)


def _chunk(fourcc, payload):
    b = fourcc + struct.pack("<I", len(payload)) + payload
    return b + (b"\0" if len(payload) & 1 else b"")


class AviWriter:
    """Writes `path + ".part"` and renames it to `path` on close(): a run that
    fails (abort(), or an exception before close) never leaves a complete-
    looking AVI under the output name, which the builders' skip-if-exists rule
    (`-n`, lib/ffmpeg.py:964-970) would then keep."""

    def __init__(self, path, w, h, rate, extradata=b"", fourcc=b"FFV1", riff_limit=RIFF_LIMIT, info=None):
        """info: RIFF INFO tags written into the header list (e.g. {b"ISFT":
        b"pixpath ffv1-gpu 8x8"}, the encoder provenance FFmpeg also writes)."""
        # unbuffered: a packet goes out as one writev of (chunk header, payload,
        # pad) straight from the caller's buffer -- no copy through a Python
        # buffer, and the GIL is released for the whole write
        self.path, self.part = path, path + ".part"
        self.info = dict(info or {})
        self.fh = open(self.part, "wb", buffering=0)
        self.w, self.h, self.rate = int(w), int(h), Fraction(rate)
        self.extradata, self.fourcc, self.limit = bytes(extradata), fourcc, riff_limit
        self.riffs = []       # per RIFF: [riff_start, movi_start, [(data_offset, size, key)]]
        self.total = 0
        self.max_size = 0
        self._write_headers()
        self._open_movi()

    # -- headers (patched on close) ------------------------------------------
    def _write_headers(self):
        self.fh.write(b"RIFF\0\0\0\0AVI ")
        us = int(round(1e6 / float(self.rate)))
        avih = struct.pack("<10I4I", us, 0, 0, 0x10 | 0x100, 0, 0, 1, 0, self.w, self.h, 0, 0, 0, 0)
        num, den = self.rate.numerator, self.rate.denominator
        strh = b"vids" + self.fourcc + struct.pack("<IHHIIIIIIiI4h", 0, 0, 0, 0, den, num, 0, 0, 0, -1, 0,
                                                    0, 0, self.w, self.h)
        bih = struct.pack("<IiiHH4sIiiII", 40 + len(self.extradata), self.w, self.h, 1, 24, self.fourcc,
                          self.w * self.h * 3, 0, 0, 0, 0)
        strf = bih + self.extradata
        indx = struct.pack("<HBBI4s3I", 4, 0, 0, 0, b"00dc", 0, 0, 0) + b"\0" * (16 * SUPER_ENTRIES)
        strl = b"strl" + _chunk(b"strh", strh) + _chunk(b"strf", strf) + _chunk(b"indx", indx)
        odml = b"odml" + _chunk(b"dmlh", b"\0" * 248)
        hdrl = b"hdrl" + _chunk(b"avih", avih) + _chunk(b"LIST", strl) + _chunk(b"LIST", odml)
        self.hdr_start = self.fh.tell()
        self.fh.write(_chunk(b"LIST", hdrl))
        if self.info:  # LIST 'INFO' (after hdrl, before movi, as avienc.c places it)
            self.fh.write(_chunk(b"LIST", b"INFO" + b"".join(_chunk(k, bytes(v) + b"\0")
                                                             for k, v in self.info.items())))
        # offsets of the fields patched on close
        base = self.hdr_start + 12
        self.off_avih = base + 8                               # avih payload
        strl_start = base + 8 + len(avih) + 8 + 4              # strl list payload after 'strl'
        self.off_strh = strl_start + 8                         # strh payload
        self.off_indx = strl_start + 8 + len(strh) + 8 + len(strf) + (len(strf) & 1) + 8
        odml_start = self.off_indx + len(indx) + 8 + 4
        self.off_dmlh = odml_start + 8

    def _open_movi(self):
        if self.riffs:
            start = self.fh.tell()
            self.fh.write(b"RIFF\0\0\0\0AVIX")
        else:
            start = 0
        movi = self.fh.tell()
        self.fh.write(b"LIST\0\0\0\0movi")
        self.riffs.append([start, movi, []])

    def _close_movi(self):
        start, movi, ents = self.riffs[-1]
        # ix00: standard index of this RIFF's packets, offsets relative to qwBaseOffset
        ix = struct.pack("<HBBI4sQI", 2, 0, 1, len(ents), b"00dc", movi, 0)
        ix += b"".join(struct.pack("<II", off - movi, size | (0 if key else 0x80000000)) for off, size, key in ents)
        ix_pos = self.fh.tell()
        self.fh.write(_chunk(b"ix00", ix))
        end = self.fh.tell()
        self._patch(movi + 4, end - movi - 8)
        self.riffs[-1].append((ix_pos, len(ix) + 8))
        if start == 0:  # idx1 (legacy index, first RIFF only): offsets relative to 'movi'
            idx1 = b"".join(struct.pack("<4sIII", b"00dc", 0x10 if key else 0, off - 8 - (movi + 8), size)
                            for off, size, key in ents)
            self.fh.write(_chunk(b"idx1", idx1))
            end = self.fh.tell()
        self._patch(start + 4, end - start - 8)

    def _patch(self, pos, value, fmt="<I"):
        cur = self.fh.tell()
        self.fh.seek(pos)
        self.fh.write(struct.pack(fmt, value))
        self.fh.seek(cur)

    def write_packet(self, data, key=True):
        """Append one packet (bytes-like; written without an extra copy)."""
        data = memoryview(data).cast("B")
        n = len(data)
        start = self.riffs[-1][0]
        if self.fh.tell() - start + n + 8 + 16 * (len(self.riffs[-1][2]) + 2) > self.limit \
                and self.riffs[-1][2]:
            self._close_movi()
            self._open_movi()
        pos = self.fh.tell()
        parts = [b"00dc" + struct.pack("<I", n), data] + ([b"\0"] if n & 1 else [])
        total = 8 + n + (n & 1)
        self._writev(parts, pos, total)
        self.riffs[-1][2].append((pos + 8, n, key))
        self.total += 1
        self.max_size = max(self.max_size, n)

    def write_packets(self, data, sizes):
        """Append len(sizes) packets held back to back in `data` (bytes-like),
        with as few writev calls as the iovec limit allows (one Python call
        per batch of packets instead of per packet)."""
        data = memoryview(data).cast("B")
        sizes = [int(n) for n in sizes]
        i, off = 0, 0
        while i < len(sizes):
            start = self.riffs[-1][0]
            pos = self.fh.tell()
            parts, ents, total, split = [], [], 0, False
            # packets of this RIFF segment (the per-packet split rule of write_packet)
            while i < len(sizes) and len(parts) < 1000:
                n = sizes[i]
                if pos + total - start + n + 8 + 16 * (len(self.riffs[-1][2]) + len(ents) + 2) > self.limit \
                        and (self.riffs[-1][2] or ents):
                    split = True
                    break
                parts.append(b"00dc" + struct.pack("<I", n))
                parts.append(data[off:off + n])
                if n & 1:
                    parts.append(b"\0")
                ents.append((pos + total + 8, n, True))
                total += 8 + n + (n & 1)
                self.max_size = max(self.max_size, n)
                off += n
                i += 1
            if ents:
                self._writev(parts, pos, total)
                self.riffs[-1][2].extend(ents)
                self.total += len(ents)
            if split:
                self._close_movi()
                self._open_movi()

    def _writev(self, parts, pos, total):
        done = 0
        while done < total:  # writev may write short
            k = os.writev(self.fh.fileno(), parts)
            done += k
            if done < total:
                rest, skip = [], k
                for b in parts:
                    b = memoryview(b).cast("B")
                    if skip >= len(b):
                        skip -= len(b)
                        continue
                    rest.append(b[skip:])
                    skip = 0
                parts = rest
        self.fh.seek(pos + total)

    def close(self):
        self._close_movi()
        first = len(self.riffs[0][2])
        # avih: dwMaxBytesPerSec, dwTotalFrames (first RIFF), dwSuggestedBufferSize
        self._patch(self.off_avih + 4, int(self.max_size * float(self.rate)))
        self._patch(self.off_avih + 16, first)
        self._patch(self.off_avih + 28, self.max_size)
        # strh: dwLength, dwSuggestedBufferSize
        self._patch(self.off_strh + 32, self.total)
        self._patch(self.off_strh + 36, self.max_size)
        self._patch(self.off_dmlh, self.total)
        # indx: one entry per RIFF's ix00
        if len(self.riffs) > SUPER_ENTRIES:
            raise ValueError("more than %d RIFF segments" % SUPER_ENTRIES)
        self._patch(self.off_indx + 4, len(self.riffs))
        for i, (_, _, ents, (ix_pos, ix_size)) in enumerate(self.riffs):
            cur = self.fh.tell()
            self.fh.seek(self.off_indx + 24 + 16 * i)
            self.fh.write(struct.pack("<QII", ix_pos, ix_size, len(ents)))
            self.fh.seek(cur)
        self.fh.close()
        os.replace(self.part, self.path)

    def abort(self):
        """Drop the partial output (the output name is never created)."""
        try:
            self.fh.close()
        finally:
            if os.path.exists(self.part):
                os.remove(self.part)


def scan(path):
    """(info, index) of an AVI without loading it: info = {w, h, rate,
    handler, fourcc, extradata} of its first VIDEO stream ('vids' strl; an
    audio strl's strh/strf never overwrite it), index = [(file offset, size)]
    of that stream's packets in file order.  Chunks are walked with seeks, so
    a tens-of-GB long-test AVPVS costs one 8-byte read per packet."""
    info, index = {}, []
    with open(path, "rb") as fh:
        fh.seek(0, 2)
        total = fh.tell()
        state = {"strl": -1, "type": None, "video": None}

        def walk(pos, end):
            while pos + 8 <= end:
                fh.seek(pos)
                hdr = fh.read(12)
                if len(hdr) < 8:
                    return
                tag, size = hdr[:4], struct.unpack_from("<I", hdr, 4)[0]
                body = pos + 8
                if tag in (b"RIFF", b"LIST"):
                    if hdr[8:12] == b"strl":
                        state["strl"] += 1
                        state["type"] = None
                    walk(body + 4, min(body + size, end))
                elif tag == b"strh":
                    fh.seek(body)
                    d = fh.read(min(size, 56))
                    state["type"] = d[:4]
                    if d[:4] == b"vids" and state["video"] is None:
                        state["video"] = state["strl"]
                        scale, rate = struct.unpack_from("<II", d, 20)
                        info["rate"] = Fraction(rate, scale)
                        info["handler"] = d[4:8]
                elif tag == b"strf":
                    if state["type"] == b"vids" and state["strl"] == state["video"] and "w" not in info:
                        fh.seek(body)
                        d = fh.read(size)
                        bi_size, w, h = struct.unpack_from("<Iii", d, 0)
                        info.update(w=w, h=abs(h), fourcc=d[16:20], extradata=d[40:bi_size])
                elif tag in (b"ISFT", b"ICMT") and tag not in info.get("tags", {}):
                    fh.seek(body)
                    info.setdefault("tags", {})[tag] = fh.read(size).rstrip(b"\0")
                elif tag[2:] in (b"dc", b"db") and tag[:2].isdigit():
                    if state["video"] is not None and int(tag[:2]) == state["video"]:
                        index.append((body, size))
                pos = body + size + (size & 1)

        walk(0, total)
    return info, index


def read_packets(path):
    """(info, packets): scan() plus the packet bytes, in order (small files / tests)."""
    info, index = scan(path)
    with open(path, "rb") as fh:
        packets = []
        for off, size in index:
            fh.seek(off)
            packets.append(fh.read(size))
    return info, packets
