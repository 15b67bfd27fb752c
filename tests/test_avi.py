"""pixpath.avi: the OpenDML AVI writer for GPU-encoded FFV1 AVPVS files and
its reader -- round trips of the packets and of the header fields, including
files split over several RIFF segments (RIFF 'AVI ' + 'AVIX').  Acceptance by
FFmpeg's demuxer is unpinned (no FFmpeg here)."""
import struct
from fractions import Fraction

import numpy as np
import pytest

from pixpath import avi


@pytest.mark.parametrize("limit", [avi.RIFF_LIMIT, 20000])
def test_round_trip(tmp_path, limit):
    rng = np.random.default_rng(1)
    pk = [rng.integers(0, 256, int(rng.integers(1, 3000)), dtype=np.uint8).tobytes() for _ in range(120)]
    extra = b"\x01\x02\x03extradata"
    path = str(tmp_path / "a.avi")
    w = avi.AviWriter(path, 1920, 1080, Fraction(60000, 1001), extradata=extra, riff_limit=limit)
    for p in pk:
        w.write_packet(p)
    w.close()
    info, got = avi.read_packets(path)
    assert got == pk
    assert (info["w"], info["h"], info["rate"], info["fourcc"], info["extradata"]) == \
        (1920, 1080, Fraction(60000, 1001), b"FFV1", extra)
    data = open(path, "rb").read()
    assert data[:4] == b"RIFF" and data[8:12] == b"AVI "
    assert struct.unpack_from("<I", data, 4)[0] + 8 <= len(data)
    riffs = data.count(b"AVIX") + 1
    if limit < avi.RIFF_LIMIT:
        assert riffs > 1
    # super index: one entry per RIFF, durations add up to the frame count
    i = data.index(b"indx") + 8
    n_used = struct.unpack_from("<I", data, i + 4)[0]
    assert n_used == riffs
    durs = [struct.unpack_from("<QII", data, i + 24 + 16 * k)[2] for k in range(n_used)]
    assert sum(durs) == len(pk)
    for k in range(n_used):  # each entry points at an ix00 chunk
        off = struct.unpack_from("<Q", data, i + 24 + 16 * k)[0]
        assert data[off:off + 4] == b"ix00"


def _two_stream_avi(path, video_first, vpk, apk, extra):
    """A hand-built AVI with a video (FFV1) and an audio (PCM) stream, as
    ffmpeg's remux of a GPU-written AVPVS with `-c:a flac/pcm` lays it out."""
    c = avi._chunk
    vstrh = b"vids" + b"FFV1" + struct.pack("<IHHIIIIIIiI4h", 0, 0, 0, 0, 1, 60, 0, len(vpk), 0, -1, 0, 0, 0, 64, 32)
    vstrf = struct.pack("<IiiHH4sIiiII", 40 + len(extra), 64, 32, 1, 24, b"FFV1", 0, 0, 0, 0, 0) + extra
    astrh = b"auds" + b"\0\0\0\0" + struct.pack("<IHHIIIIIIiI4h", 0, 0, 0, 0, 1, 48000, 0, 0, 0, -1, 4, 0, 0, 0, 0)
    astrf = struct.pack("<HHIIHH", 1, 2, 48000, 192000, 4, 16)  # WAVEFORMATEX: w/h/fourcc would read garbage
    vl = c(b"LIST", b"strl" + c(b"strh", vstrh) + c(b"strf", vstrf))
    al = c(b"LIST", b"strl" + c(b"strh", astrh) + c(b"strf", astrf))
    vid, aid = (b"00", b"01") if video_first else (b"01", b"00")
    hdrl = c(b"LIST", b"hdrl" + c(b"avih", b"\0" * 56) + (vl + al if video_first else al + vl))
    movi = b"movi"
    for v, a in zip(vpk, apk):
        movi += c(vid + b"dc", v) + c(aid + b"wb", a)
    body = b"AVI " + hdrl + c(b"LIST", movi)
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", len(body)) + body)


@pytest.mark.parametrize("video_first", [True, False])
def test_two_stream_avi_takes_the_video_stream(tmp_path, video_first):
    rng = np.random.default_rng(2)
    vpk = [rng.integers(0, 256, int(rng.integers(1, 500)), dtype=np.uint8).tobytes() for _ in range(9)]
    apk = [rng.integers(0, 256, 3200, dtype=np.uint8).tobytes() for _ in range(9)]
    extra = b"cfgrecord"
    path = str(tmp_path / "av.avi")
    _two_stream_avi(path, video_first, vpk, apk, extra)
    info, got = avi.read_packets(path)
    assert got == vpk
    assert (info["w"], info["h"], info["rate"], info["fourcc"], info["extradata"]) == (64, 32, Fraction(60), b"FFV1",
                                                                                        extra)
    info2, index = avi.scan(path)
    assert [s for _, s in index] == [len(p) for p in vpk]


def test_info_tag_and_atomic_output(tmp_path):
    """The encoder provenance (RIFF INFO ISFT) round trips; the file appears
    under its name only on close(), and abort() leaves nothing behind (the
    builders' skip-if-exists rule never sees a partial AVPVS)."""
    import os
    path = str(tmp_path / "p.avi")
    w = avi.AviWriter(path, 64, 32, 60, extradata=b"x", info={b"ISFT": b"pixpath ffv1-gpu v3 intra 8x8 slices"})
    w.write_packet(b"abc")
    assert not os.path.exists(path) and os.path.exists(path + ".part")
    w.close()
    info, pk = avi.read_packets(path)
    assert pk == [b"abc"] and info["tags"][b"ISFT"] == b"pixpath ffv1-gpu v3 intra 8x8 slices"
    assert not os.path.exists(path + ".part")
    bad = str(tmp_path / "bad.avi")
    w = avi.AviWriter(bad, 64, 32, 60)
    w.write_packet(b"abc")
    w.abort()
    assert not os.path.exists(bad) and not os.path.exists(bad + ".part")


@pytest.mark.parametrize("limit", [avi.RIFF_LIMIT, 20000])
def test_batched_writes_equal_per_packet_writes(tmp_path, limit):
    """write_packets (one writev per up to ~330 packets) lays out exactly the
    file write_packet does, RIFF splits included."""
    rng = np.random.default_rng(3)
    sizes = [int(rng.integers(1, 3000)) for _ in range(700)]
    data = rng.integers(0, 256, sum(sizes), dtype=np.uint8)
    a, b = str(tmp_path / "a.avi"), str(tmp_path / "b.avi")
    w = avi.AviWriter(a, 64, 32, 60, extradata=b"e", riff_limit=limit)
    off = 0
    for n in sizes:
        w.write_packet(data[off:off + n])
        off += n
    w.close()
    w = avi.AviWriter(b, 64, 32, 60, extradata=b"e", riff_limit=limit)
    w.write_packets(data[:sizes[0] + sizes[1]], sizes[:2])
    w.write_packets(data[sizes[0] + sizes[1]:], sizes[2:])
    w.close()
    assert open(a, "rb").read() == open(b, "rb").read()
