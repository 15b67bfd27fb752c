"""pixpath.io.LumaReader (the SI/TI hook's luma-only decode) on CPU: the luma
plane of every frame of Y4M / raw files, identical to the full-frame reader's
first plane, whether the file is seekable or a pipe."""
import os

import numpy as np
import pytest

import pyoracle as po
import synth
from pixpath import io as pio


def _write(path, fmt_name, fmt, n, w, h):
    frames = [synth.smooth_frame(t, fmt, w, h) for t in range(n)]
    if path.endswith(".y4m"):
        wr = pio.Y4MWriter(path, fmt_name, w, h, 60)
    else:
        wr = pio.RawWriter(path)
    for f in frames:
        wr.write(pio.join_planes(synth.batch([f])))
    wr.close()
    return np.stack([f[0] for f in frames])


@pytest.mark.parametrize("ext,fmt_name,fmt", [(".y4m", "yuv422p10le", po.YUV422P10LE), (".y4m", "yuv420p", po.YUV420P),
                                               (".raw", "yuv420p10le", po.YUV420P10LE)])
@pytest.mark.parametrize("k", [1, 4, 16])
def test_luma_reader_matches_full_frames(tmp_path, ext, fmt_name, fmt, k):
    w, h, n = 96, 54, 11
    path = str(tmp_path / ("clip" + ext))
    luma = _write(path, fmt_name, fmt, n, w, h)
    rd = pio.LumaReader(path, f=fmt_name, w=w, h=h)
    assert (rd.w, rd.h, rd.depth) == (w, h, 10 if "10" in fmt_name else 8)
    dt = np.uint16 if rd.depth > 8 else np.uint8
    got = []
    buf = np.empty((k, rd.luma_bytes), np.uint8)
    while True:
        m = rd.read_into(buf, k)
        got.extend(buf[i].view(dt).reshape(h, w).copy() for i in range(m))
        if m < k:
            break
    rd.close()
    np.testing.assert_array_equal(np.stack(got), luma)


def test_luma_reader_from_a_pipe(tmp_path):
    """A non-seekable input (the ffmpeg decode pipe case) reads past chroma."""
    w, h, n = 64, 36, 5
    path = str(tmp_path / "clip.y4m")
    luma = _write(path, "yuv422p10le", po.YUV422P10LE, n, w, h)
    r, wfd = os.pipe()
    data = open(path, "rb").read()
    import threading

    def feed():
        with os.fdopen(wfd, "wb") as f:
            f.write(data)
    t = threading.Thread(target=feed)
    t.start()
    rd = pio.LumaReader(os.fdopen(r, "rb"))
    assert not rd.seekable
    buf = np.empty((n + 1, rd.luma_bytes), np.uint8)
    assert rd.read_into(buf, n + 1) == n
    rd.close()
    t.join()
    np.testing.assert_array_equal(buf[:n].view(np.uint16).reshape(n, h, w), luma)
