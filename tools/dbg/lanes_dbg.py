# debug: AVPVS writer lanes (split 1 vs 3) -- which packets differ
import sys, os
sys.path.insert(0, "processing-chain_amd"); sys.path.insert(0, "tests"); sys.path.insert(0, "oracle")
import numpy as np, torch
import pyoracle as po, synth
from pixpath import avi, ffv1
from pixpath.frames import FrameBatch
gpu = torch.device("cuda", 0)
w, h, n = 320, 180, 25
frames = [synth.smooth_frame(i, po.YUV422P10LE, w, h) for i in range(n)]
src = FrameBatch.interleaved("yuv422p10le", w, h, n, device=gpu)
for i, f in enumerate(frames):
    for p in range(3):
        src.view(p)[i].copy_(torch.from_numpy(f[p].astype(np.uint16)))
res = {}
for k in (1, 3):
    path = "/tmp/lanes_%d.avi" % k
    wr = ffv1.Ffv1AviWriter(path, "yuv422p10le", w, h, 60, slices=(4, 4), batch=10, device=gpu, split=k)
    for a, b in ((0, 3), (3, 11), (11, 12), (12, 25)):
        wr.write_device(FrameBatch.interleaved("yuv422p10le", w, h, b - a, device=gpu, storage=src.storage[a:b]))
    wr.close()
    info, pk = avi.read_packets(path)
    res[k] = pk
    print(k, os.path.getsize(path), len(pk), [len(x) for x in pk])
for i, (x, y) in enumerate(zip(res[1], res[3])):
    if x != y:
        print("packet", i, "differs", len(x), len(y))
