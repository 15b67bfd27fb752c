#!/usr/bin/env python3
"""Isolated launches of the bench kernels (config 2 shapes) for rocprofv3 counter passes.

  python3 tools/prof_kernels.py [--which scale|siti|both] [--launches 3] [--frames 600]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "processing-chain_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="both")
    ap.add_argument("--launches", type=int, default=3)
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--flags", default="lanczos")
    ap.add_argument("--src", default="yuv422p10le:1280x720", help="source fmt:WxH (config 3: yuv420p:3840x2160)")
    a = ap.parse_args()
    import torch
    from pixpath import ops
    from pixpath.frames import FrameBatch
    dev = torch.device("cuda", 0)
    n = a.frames
    g = torch.Generator(device=dev)
    g.manual_seed(910)
    if a.which in ("scale", "both"):
        sfmt, wh = a.src.split(":")
        sw, sh = (int(t) for t in wh.split("x"))
        hi = 941 if "10" in sfmt else 236
        src = FrameBatch(sfmt, sw, sh, n, device=dev)
        for p in range(3):
            v = src.view(p)
            v.copy_(torch.randint(16, hi, v.shape, generator=g, device=dev, dtype=torch.int32).to(v.dtype))
        dst = FrameBatch("yuv422p10le", 1920, 1080, n, device=dev)
        sc = ops.Scaler(sfmt, sw, sh, "yuv422p10le", 1920, 1080, flags=a.flags)
        for _ in range(a.launches):
            sc(src, dst)
        torch.cuda.synchronize()
        del src, dst
    if a.which in ("siti", "both"):
        luma = torch.randint(64, 941, (n, 1080, 1920), generator=g, device=dev, dtype=torch.int32).to(torch.uint16)
        for _ in range(a.launches):
            ops.siti(luma, 10)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
