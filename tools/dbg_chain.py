"""Debug: one chain case through the library at PIXPATH_LIB vs the oracle; mismatch pattern."""
import sys, os
import numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "oracle"); sys.path.insert(0, "processing-chain_amd")
import pyoracle as po, synth
from pixpath import ops
from pixpath.frames import FrameBatch
sf, sw, sh, df, dw, dh = po.YUV420P, 1280, 720, po.YUV422P, 1920, 1080
rng = np.random.default_rng(sw + dh)
frames = [synth.noise_frame(rng, sf, sw, sh)]
src = FrameBatch.from_numpy(sf, synth.batch(frames), device="cuda:0")
sc = ops.Scaler(sf, sw, sh, df, dw, dh, flags="bicubic", chain=True)
out = sc(src).to_numpy()
mid = po.scale(sf, frames[0], po.YUV420P, dw, dh, po.SWS_BICUBIC)
ref = po.scale(po.YUV420P, mid, df, dw, dh, po.SWS_BICUBIC)
for p in range(3):
    bad = np.argwhere(out[p][0] != ref[p])
    print(os.environ.get("TAG"), "plane", p, "mismatches", len(bad), "shape", ref[p].shape)
    if len(bad):
        rows = np.unique(bad[:, 0]); cols = np.unique(bad[:, 1])
        print("  rows", rows[:20], "... n", len(rows), " cols", cols[:20], "... n", len(cols))
        d = out[p][0].astype(int) - ref[p].astype(int)
        print("  diff range", d.min(), d.max(), "sample", [(int(r), int(c), int(out[p][0][r, c]), int(ref[p][r, c])) for r, c in bad[:6]])
