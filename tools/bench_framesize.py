#!/usr/bin/env python3
"""Throughput of the p02 frame-size scanner.

Host-only work: libpixpath's pp_annexb_frame_sizes / pp_ivf_frame_sizes
(csrc/scan.cpp) over synthetic Annex-B H.264 and IVF streams shaped like a
batch of p01 segments (600 frames of ~20 kB each per 10 s segment), timed on
bytes resident in host memory, next to the byte-at-a-time restatement of the
reference's loop (oracle/framesize_ref.py, the `port` baseline) on a bounded
sample.  Prints one JSON line.

  python tools/bench_framesize.py [--segments 64] [--port-mb 2]
"""
import argparse
import json
import os
import struct
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "processing-chain_amd"), os.path.join(ROOT, "oracle")]

from pixpath import framesize  # noqa: E402


def h264_segments(rng, segments, frames=600, mean=20000):
    """Start code + NAL header + zero-free payload per frame (SPS/PPS per segment)."""
    sizes = np.maximum(16, rng.exponential(mean, segments * frames).astype(np.int64))
    total = int(sizes.sum()) + segments * frames * 5 + segments * 32
    buf = rng.integers(1, 256, total, dtype=np.uint8)
    pos = 0
    for s in range(segments):
        for hdr in (0x67, 0x68):
            buf[pos:pos + 5] = [0, 0, 0, 1, hdr]
            pos += 16
        for f in range(frames):
            buf[pos:pos + 5] = [0, 0, 0, 1, 0x65 if f == 0 else 0x41]
            pos += 5 + int(sizes[s * frames + f])
    return buf[:pos]


def ivf_stream(rng, frames, mean=20000):
    sizes = np.maximum(4, rng.exponential(mean, frames).astype(np.int64))
    out = bytearray(b"DKIF" + struct.pack("<HHIHHIIII", 0, 32, 0x30395056, 1920, 1080, 60, 1, frames, 0))
    body = rng.integers(0, 256, int(sizes.sum()), dtype=np.uint8)
    body_off = 0
    parts = [bytes(out)]
    for i, n in enumerate(sizes.tolist()):
        chunk = body[body_off:body_off + n].copy()
        chunk[0] = 0x82
        body_off += n
        parts.append(struct.pack("<IQ", n, i) + chunk.tobytes())
    return np.frombuffer(b"".join(parts), dtype=np.uint8)


def rate(fn, nbytes, min_s=1.0):
    fn()
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += 1
        dt = time.perf_counter() - t0
        if dt >= min_s:
            return nbytes * n / dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segments", type=int, default=64)
    ap.add_argument("--port-mb", type=float, default=2.0)
    args = ap.parse_args()
    import framesize_ref as ref

    rng = np.random.default_rng(20)
    h264 = h264_segments(rng, args.segments)
    ivf = ivf_stream(rng, args.segments * 600)
    n_frames = len(framesize.annexb_frame_sizes(h264, "h264"))
    native_h264 = rate(lambda: framesize.annexb_frame_sizes(h264, "h264"), h264.size)
    native_h265 = rate(lambda: framesize.annexb_frame_sizes(h264, "h265"), h264.size)
    native_ivf = rate(lambda: framesize.ivf_frame_sizes(ivf), ivf.size)
    sample = h264[: int(args.port_mb * 2 ** 20)].tobytes()
    t0 = time.perf_counter()
    port_sizes = ref.annexb_sizes(sample, "h264")
    port = len(sample) / (time.perf_counter() - t0)
    assert port_sizes[:-1] == framesize.annexb_frame_sizes(np.frombuffer(sample, np.uint8), "h264")[:-1]
    mb = 2.0 ** 20
    print(json.dumps({
        "metric": "p02 frame-size scan (lib/get_framesize.py) bytes/s, host", "unit": "MB/s",
        "value": round(native_h264 / mb, 1), "h265_mb_s": round(native_h265 / mb, 1),
        "ivf_mb_s": round(native_ivf / mb, 1), "threads": 1,
        "workload": {"segments": args.segments, "frames": n_frames, "h264_bytes": int(h264.size),
                     "ivf_bytes": int(ivf.size), "resident": "host memory (file read excluded)"},
        "cpu_baseline": {"kind": "port", "value": round(port / mb, 3), "unit": "MB/s", "cores": 1,
                         "sample": "%.1f MB of the same H.264 stream through oracle/framesize_ref.py "
                                   "(the reference's per-byte loop on ints)" % (len(sample) / mb)},
        "speedup_vs_port": round(native_h264 / port, 1),
    }))


if __name__ == "__main__":
    main()
