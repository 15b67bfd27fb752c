import sys, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "oracle"); sys.path.insert(0, "processing-chain_amd")
import pyoracle as po, synth
from pixpath import ops
from pixpath.frames import FrameBatch
import torch
gpu = torch.device("cuda", 0)
for fmt, w, h, W, H in [(po.YUV420P, 1920, 800, 1920, 1080), (po.YUV420P, 1920, 1080, 1920, 1080), (po.YUV420P10LE, 1920, 1080, 1920, 1080), (po.YUV422P, 1920, 1012, 1920, 1080)]:
    rng = np.random.default_rng(8)
    frames = [synth.noise_frame(rng, fmt, w, h) for _ in range(1)]
    src = FrameBatch.from_numpy(fmt, synth.batch(frames), device=gpu)
    out = ops.cpvs(src, W, H).to_numpy()[0][0]
    padded = po.pad(fmt, frames[0], W, H, (W - w) // 2, (H - h) // 2)
    if po.fmt_info(fmt)[0] == 8:
        (ref,) = po.scale(fmt, padded, po.UYVY422, W, H)
    else:
        ref = po.v210_pack(po.scale(fmt, padded, po.YUV422P10LE, W, H))
    out = out.reshape(ref.shape)
    bad = np.argwhere(out != ref)
    print(fmt, w, h, "mismatches", len(bad))
    if len(bad):
        rows = np.unique(bad[:, 0]); print(" rows", rows[:20], len(rows))
        print(" cols mod 4", np.bincount(bad[:, 1] % 4, minlength=4), "first", bad[:5].tolist())
        r, c = bad[0]; print(" got", out[r, c:c+16].tolist(), "ref", ref[r, c:c+16].tolist())
