"""Streaming pipeline (pixpath.pipeline): pinned double buffers, two streams.

Frames through the pipeline equal the scaler run directly; a failing writer
(an encoder that died) makes run() raise instead of hanging."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class MemReader:
    def __init__(self, frames):
        self.frames, self.i = frames, 0

    def read_into(self, buf, n):
        b = np.frombuffer(buf, np.uint8).reshape(-1, self.frames.shape[1])
        k = min(n, len(self.frames) - self.i)
        b[:k] = self.frames[self.i:self.i + k]
        self.i += k
        return k


class ListWriter:
    def __init__(self):
        self.out = []

    def write(self, fr):
        self.out.append(np.array(np.frombuffer(memoryview(fr).cast("B"), np.uint8)))


class FailingWriter:
    def __init__(self, after):
        self.after, self.n = after, 0

    def write(self, fr):
        self.n += 1
        if self.n > self.after:
            raise BrokenPipeError("encoder exited")


def _stage(gpu):
    from pixpath import ops
    from pixpath.pipeline import Stage
    sc = ops.Scaler("yuv420p", 64, 48, "yuv422p10le", 96, 72, flags="bicubic")
    return sc, Stage("yuv420p", 64, 48, "yuv422p10le", 96, 72, lambda s, d, st: sc(s, d, stream=st))


def _frames(n):
    from pixpath import formats
    fb = formats.frame_bytes("yuv420p", 64, 48)
    return np.random.default_rng(5).integers(0, 256, (n, fb), dtype=np.uint8)


def test_pipeline_matches_direct(gpu):
    import torch
    from pixpath import io as pio
    from pixpath.frames import FrameBatch
    from pixpath.pipeline import Pipeline
    sc, stage = _stage(gpu)
    frames = _frames(23)
    w = ListWriter()
    n = Pipeline(stage, batch=8, device=0).run(MemReader(frames), w)
    assert n == 23
    got = np.concatenate([o.reshape(-1) for o in w.out])
    planes = pio.split_planes(frames, "yuv420p", 64, 48)
    ref = sc(FrameBatch.from_numpy("yuv420p", planes, device=gpu)).to_numpy()
    torch.cuda.synchronize()
    assert np.array_equal(got, pio.join_planes(ref).reshape(-1))


def test_pipeline_writer_failure_raises(gpu):
    from pixpath.pipeline import Pipeline
    _, stage = _stage(gpu)
    res = {}

    def run():
        try:
            Pipeline(stage, batch=4, device=0).run(MemReader(_frames(40)), FailingWriter(after=1))
        except BrokenPipeError as e:
            res["err"] = e
    t = threading.Thread(target=run, daemon=True)
    t.start()
    t.join(timeout=60)
    assert not t.is_alive(), "pipeline hung after a writer failure"
    assert "err" in res
