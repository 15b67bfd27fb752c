"""GPU experiment: SI/TI of the same noise under different layouts (debug aid)."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "processing-chain_amd"), os.path.join(ROOT, "oracle")]
import siti_ref
from pixpath import ops

def run(frames, depth, pitch=None, off=0):
    n, h, w = frames.shape
    dt = np.uint16 if depth > 8 else np.uint8
    P = pitch or w
    big = np.zeros((n, h, P + off), dt)
    big[:, :, off:off + w] = frames
    t = torch.from_numpy(big).cuda()[:, :, off:off + w]
    si, ti = ops.siti(t, depth)
    torch.cuda.synchronize()
    return si.cpu().numpy(), ti.cpu().numpy()

rng = np.random.default_rng(1)
for (w, h) in [(3, 3), (3, 16), (3, 17), (16, 3), (497, 37), (496, 37), (497, 32), (8, 18)]:
    for depth in (8, 10):
        hi = 235 if depth == 8 else 940
        fr = rng.integers(16, hi + 1, (4, h, w)).astype(np.uint16 if depth > 8 else np.uint8)
        rsi, rti = siti_ref.siti(fr)
        res = []
        for name, kw in [("contig", {}), ("pitch64", {"pitch": (w + 63) // 64 * 64}), ("off1", {"pitch": w + 8, "off": 1})]:
            si, ti = run(fr, depth, **kw)
            ok_si = np.allclose(si, rsi, rtol=1e-4, atol=1e-9)
            ok_ti = np.allclose(ti[1:], rti[1:], rtol=1e-12, atol=1e-12)
            res.append("%s:%s%s" % (name, "S" if ok_si else "s!", "T" if ok_ti else "t!"))
        print(w, h, depth, " ".join(res), flush=True)
