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
