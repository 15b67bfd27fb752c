#!/usr/bin/env python3
"""Timing of the create_avpvs_segment chain plan vs its two stages alone (HIP
events, 600-frame launches): measurement only.

  python3 tools/chain_ablate.py [--frames 600] [--src yuv420p10le] [--dst yuv422p10le]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "processing-chain_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--src", default="yuv420p10le")
    ap.add_argument("--dst", default="yuv422p10le")
    ap.add_argument("--size", default="1280x720")
    a = ap.parse_args()
    import torch
    from pixpath import ops
    from pixpath.frames import FrameBatch
    dev = torch.device("cuda", 0)
    n = a.frames
    sw, sh = (int(v) for v in a.size.split("x"))
    src = FrameBatch(a.src, sw, sh, n, device=dev)
    for p in range(3):
        v = src.view(p)
        v.copy_(torch.randint(0, (1 << src.fmt.depth), v.shape, device=dev, dtype=torch.int32).to(v.dtype))
    mid = FrameBatch("yuv420p", 1920, 1080, n, device=dev)
    dst = FrameBatch(a.dst, 1920, 1080, n, device=dev)

    def timed(fn, k=5):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(k):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / k

    chain = ops.Scaler(a.src, sw, sh, a.dst, 1920, 1080, chain=True)
    s1 = ops.Scaler(a.src, sw, sh, "yuv420p", 1920, 1080)
    s2 = ops.Scaler("yuv420p", 1920, 1080, a.dst, 1920, 1080)
    res = {"chain_ms": timed(lambda: chain(src, dst)), "chain_path": chain.kernel_path, "chain_stats": chain.stats,
           "stage1_ms": timed(lambda: s1(src, mid)), "stage1_stats": s1.stats,
           "stage2_ms": timed(lambda: s2(mid, dst)), "stage2_path": s2.kernel_path,
           "env": {k: v for k, v in os.environ.items() if k.startswith("PIXPATH_")}}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
