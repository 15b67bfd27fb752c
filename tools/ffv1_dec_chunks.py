"""FFV1 decoder: one 600-frame launch against the same frames decoded in
sequential launches of K frames (measurement only).  A launch of K frames has
K x 64 slice chains whose hot context states (~8 KB per slice on the bench
content) are K x 0.5 MB: fewer frames per launch keep them in the 256-MB
Infinity Cache at the price of fewer chains in flight.  Prints one JSON line
per K: total decode ms for the 600 frames."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "processing-chain_amd"))


def main():
    import numpy as np
    import torch
    from pixpath import ffv1
    from pixpath.frames import FrameBatch
    dev = torch.device("cuda", 0)
    w, h, n = 1920, 1080, 600
    src = FrameBatch("yuv422p10le", w, h, n, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(910)
    fr = torch.arange(n, device=dev, dtype=torch.int32).view(n, 1, 1)
    for p in range(3):  # bench.py bench_ffv1's content
        v = src.view(p)
        yy = torch.arange(v.shape[1], device=dev, dtype=torch.int32).view(1, -1, 1)
        xx = torch.arange(v.shape[2], device=dev, dtype=torch.int32).view(1, 1, -1)
        noise = torch.randint(-4, 5, v.shape, generator=g, device=dev, dtype=torch.int32)
        v.copy_(((xx * (p + 1) + yy * 2 + 3 * fr) % 800 + 100 + noise).clamp(64, 940).to(v.dtype))
    enc = ffv1.Ffv1Encoder("yuv422p10le", w, h, slices=(8, 8), max_frames=n, device=dev)
    buf, sizes = enc.encode(src)
    pk = buf.cpu().pin_memory().numpy()
    sizes = np.asarray(sizes, dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(sizes)])
    dec = ffv1.Ffv1Decoder(enc.extradata, w, h, max_frames=n, device=dev)
    ks = [int(a) for a in sys.argv[1:]] or [600, 300, 200, 150, 100, 60]
    for K in ks:
        outs = [FrameBatch("yuv422p10le", w, h, min(K, n - k0), device=dev) for k0 in range(0, n, K)]

        def run():
            for i, k0 in enumerate(range(0, n, K)):
                k1 = min(n, k0 + K)
                dec.decode(pk[offs[k0]:offs[k1]], sizes[k0:k1], dst=outs[i])
        run()
        torch.cuda.synchronize()
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            run()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        ok = all(bool(torch.equal(outs[i].view(p), src.view(p)[k0:k0 + outs[i].n]))
                 for i, k0 in enumerate(range(0, n, K)) for p in range(3))
        print(json.dumps({"frames_per_launch": K, "decode_ms_600": round(ms, 2),
                          "frames_per_s": round(n / ms * 1e3, 1), "lossless": ok}), flush=True)


if __name__ == "__main__":
    main()
