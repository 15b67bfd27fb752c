"""FFV1 encoder / decoder timing on content of different context statistics
(measurement only): constant frames (one context), moving gradients + noise
(bench content), uniform noise (every context); 8x8 and 16x16 slices.
Prints one JSON line per case: encode / decode ms per 600-frame batch."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "processing-chain_amd"))


def main():
    import torch
    from pixpath import ffv1
    from pixpath.frames import FrameBatch
    dev = torch.device("cuda", 0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 600
    src = FrameBatch("yuv422p10le", 1920, 1080, n, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    for content in ("constant", "gradient", "noise"):
        fr = torch.arange(n, device=dev, dtype=torch.int32).view(n, 1, 1)
        for p in range(3):
            v = src.view(p)
            if content == "constant":
                v.fill_(512)
            elif content == "noise":
                v.copy_(torch.randint(64, 941, v.shape, generator=g, device=dev, dtype=torch.int32).to(v.dtype))
            else:
                yy = torch.arange(v.shape[1], device=dev, dtype=torch.int32).view(1, -1, 1)
                xx = torch.arange(v.shape[2], device=dev, dtype=torch.int32).view(1, 1, -1)
                noise = torch.randint(-4, 5, v.shape, generator=g, device=dev, dtype=torch.int32)
                v.copy_(((xx * (p + 1) + yy * 2 + 3 * fr) % 800 + 100 + noise).clamp(64, 940).to(v.dtype))
        for grid in ((8, 8), (16, 16)):
            enc = ffv1.Ffv1Encoder("yuv422p10le", 1920, 1080, slices=grid, max_frames=n, device=dev)
            buf, sizes = enc.encode(src)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(2):
                buf, sizes = enc.encode(src)
            torch.cuda.synchronize()
            te = (time.perf_counter() - t0) / 2
            pk = buf.cpu().numpy()
            dec = ffv1.Ffv1Decoder(enc.extradata, 1920, 1080, max_frames=n, device=dev)
            out = FrameBatch("yuv422p10le", 1920, 1080, n, device=dev)
            dec.decode(pk, sizes, dst=out)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(2):
                dec.decode(pk, sizes, dst=out)
            torch.cuda.synchronize()
            td = (time.perf_counter() - t0) / 2
            ok = all(bool(torch.equal(out.view(p), src.view(p))) for p in range(3))
            print(json.dumps({"content": content, "slices": list(grid), "frames": n, "encode_ms": round(te * 1e3, 2),
                              "decode_ms": round(td * 1e3, 2), "bytes_per_frame": round(float(sizes.mean()), 1),
                              "lossless": ok}), flush=True)
            del enc, dec


if __name__ == "__main__":
    main()
