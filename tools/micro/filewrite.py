"""Write-path micro for the AVPVS writer: ~1 GB of packets (600 x 1.67 MB,
the e2e bench's single PVS) appended to a fresh file as (a) os.writev of
(header, payload) parts -- pixpath.avi today -- and (b) posix_fallocate +
mmap of the range + copies by T threads (numpy copies release the GIL).
usage: python tools/micro/filewrite.py [dir]"""
import mmap
import os
import sys
import tempfile
import threading
import time

import numpy as np

d = sys.argv[1] if len(sys.argv) > 1 else tempfile.gettempdir()
n, size = 600, 1_673_427
src = np.random.default_rng(1).integers(0, 255, n * size, dtype=np.uint8)
hdr = [b"00dc" + int(size).to_bytes(4, "little") for _ in range(n)]


def writev(path):
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    t0 = time.perf_counter()
    for b in range(0, n, 300):
        parts = []
        for i in range(b, min(n, b + 300)):
            parts += [hdr[i], memoryview(src[i * size:(i + 1) * size])]
        os.writev(fd, parts)
    dt = time.perf_counter() - t0
    os.close(fd)
    return dt


def mm(path, T):
    fd = os.open(path, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o644)
    t0 = time.perf_counter()
    pos = 0
    for b in range(0, n, 300):
        k = min(n, b + 300) - b
        total = k * (8 + size)
        os.posix_fallocate(fd, pos, total)
        lo = pos & ~(mmap.ALLOCATIONGRANULARITY - 1)
        m = mmap.mmap(fd, pos + total - lo, offset=lo)
        dst = np.frombuffer(m, np.uint8)
        base = pos - lo

        def work(t):
            for j in range(t, k, T):
                o = base + j * (8 + size)
                dst[o:o + 8] = np.frombuffer(hdr[b + j], np.uint8)
                dst[o + 8:o + 8 + size] = src[(b + j) * size:(b + j + 1) * size]
        ths = [threading.Thread(target=work, args=(t,)) for t in range(T)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        del dst
        m.close()
        pos += total
    dt = time.perf_counter() - t0
    os.close(fd)
    return dt


for rep in range(3):
    for name, fn in (("writev", writev), ("mmap1", lambda p: mm(p, 1)), ("mmap4", lambda p: mm(p, 4)),
                     ("mmap8", lambda p: mm(p, 8))):
        p = os.path.join(d, "fw_%s.bin" % name)
        dt = fn(p)
        print("%s %.1f ms %.2f GB/s" % (name, dt * 1e3, n * size / dt / 1e9), flush=True)
        os.remove(p)
