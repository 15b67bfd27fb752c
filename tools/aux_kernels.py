#!/usr/bin/env python3
"""HIP-event timing + HBM roofline of the non-scaler kernels (cpvs, v210, pad,
stall compose) at the CPVS/AVPVS shapes of the bench configs.

  python3 tools/aux_kernels.py [--frames 600] [--launches 5] [--out profiles/r2/aux_kernels.json]

Algorithmic bytes per launch = bytes every output frame must read + write
(source planes it depends on, once; the packed/padded output, once).  Peak =
8 TB/s (MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "processing-chain_amd"))
PEAK = 8.0e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    from pixpath import formats, ops, spinner
    from pixpath.frames import FrameBatch
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(355)
    n = a.frames

    def filled(fmt, w, h, k):
        fb = FrameBatch(fmt, w, h, k, device=dev)
        hi = (1 << fb.fmt.depth) - 1
        for p in range(len(fb.planes)):
            v = fb.view(p)
            v.copy_(torch.randint(0, hi + 1, v.shape, generator=g, device=dev, dtype=torch.int32).to(v.dtype))
        return fb

    def plane_bytes(fb):
        return sum(fb.view(p).numel() * fb.view(p).element_size() for p in range(len(fb.planes)))

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.launches):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return sum(ts) / len(ts)

    rows = []

    def report(name, kernel, ms, rd, wr, note):
        ach = (rd + wr) / (ms * 1e-3)
        rows.append({"case": name, "kernel": kernel, "frames": n, "avg_launch_ms": round(ms, 4),
                     "bytes_read": rd, "bytes_written": wr, "achieved_GBps": round(ach / 1e9, 1),
                     "frac_of_8TBps": round(ach / PEAK, 4), "note": note})
        print(json.dumps(rows[-1]), flush=True)

    # PC CPVS of a 10-bit AVPVS (config 1/2/4 display size): yuv422p10le 1080p -> v210
    src = filled("yuv422p10le", 1920, 1080, n)
    dst = FrameBatch(formats.V210, 1920, 1080, n, device=dev)
    ms = timed(lambda: ops.cpvs(src, dst=dst))
    report("cpvs_v210_1080p", "cpvs_kernel<10,false>", ms, plane_bytes(src), plane_bytes(dst),
           "fps=60 (identity) + pad no-op + v210")
    ms = timed(lambda: ops.v210_pack(src, dst=dst))
    report("v210_pack_1080p", "cpvs_kernel<10,false>", ms, plane_bytes(src), plane_bytes(dst), "pp_v210_pack (the CPVS kernel, zero pad)")
    del dst
    # stall compose: 1080p 10-bit output frames of one frozen frame + spinner
    anim, _ = spinner.load_apng(os.path.join(ROOT, "tests", "golden", "spinner-128-white.png"))
    ops.spinner_upload(anim, "yuv422p10le", device=dev)
    import numpy as np
    si = np.zeros(n, np.int32)
    sp = (np.arange(n) % len(anim)).astype(np.int32)
    one = FrameBatch("yuv422p10le", 1920, 1080, 1, device=dev)
    for p in range(3):
        one.planes[p].copy_(src.planes[p][:1])
    out = FrameBatch("yuv422p10le", 1920, 1080, n, device=dev)
    ms = timed(lambda: ops.stall_compose(one, si, sp, dst=out))
    report("stall_1080p10", "stall_kernel", ms, plane_bytes(one), plane_bytes(out),
           "output frames of one frozen frame + animated spinner (source read once from HBM, then L2/MALL)")
    del out, src
    # pad: 1280x720 AVPVS on a 1920x1080 canvas (10-bit 4:2:2)
    s720 = filled("yuv422p10le", 1280, 720, n)
    d1080 = FrameBatch("yuv422p10le", 1920, 1080, n, device=dev)
    ms = timed(lambda: ops.pad(s720, 1920, 1080, dst=d1080))
    report("pad_720p_to_1080p10", "pad_kernel", ms, plane_bytes(s720), plane_bytes(d1080), "vf_pad centring")
    dv = FrameBatch(formats.V210, 1920, 1080, n, device=dev)
    ms = timed(lambda: ops.cpvs(s720, 1920, 1080, dst=dv))
    report("cpvs_v210_720p_on_1080p", "cpvs_kernel<10,false>", ms, plane_bytes(s720), plane_bytes(dv),
           "pad + v210 fused")
    del s720, d1080, dv
    # PC CPVS of an 8-bit 4:2:0 AVPVS: yuv420p 1080p -> uyvy422 (bicubic chroma 2x)
    s8 = filled("yuv420p", 1920, 1080, n)
    du = FrameBatch(formats.UYVY422, 1920, 1080, n, device=dev)
    ms = timed(lambda: ops.cpvs(s8, dst=du))
    report("cpvs_uyvy_420p_1080p", "cpvs_kernel<8,true>", ms, plane_bytes(s8), plane_bytes(du),
           "4:2:0 -> 4:2:2 bicubic + uyvy422")
    del s8, du
    # 10-bit 4:2:0 AVPVS -> v210 (4:2:0 -> 4:2:2 bicubic + v210)
    s10 = filled("yuv420p10le", 1920, 1080, n)
    dv = FrameBatch(formats.V210, 1920, 1080, n, device=dev)
    ms = timed(lambda: ops.cpvs(s10, dst=dv))
    report("cpvs_v210_420p10_1080p", "cpvs_kernel<10,true>", ms, plane_bytes(s10), plane_bytes(dv),
           "4:2:0 -> 4:2:2 bicubic + v210")
    del s10, dv
    # long-test canvas (create_avpvs_segment): 720p yuv420p10le segment -> overlay yuv420p -> yuv422p10le 1080p
    c720 = filled("yuv420p10le", 1280, 720, n)
    c1080 = FrameBatch("yuv422p10le", 1920, 1080, n, device=dev)
    chain = ops.Scaler("yuv420p10le", 1280, 720, "yuv422p10le", 1920, 1080, flags="bicubic", chain=True)
    ms = timed(lambda: chain(c720, c1080))
    report("chain_720p10_to_1080p422p10", "strip_kernel<u16,8,..,FUSE=10>" if chain.kernel_path else "two launches",
           ms, plane_bytes(c720), plane_bytes(c1080), "scale -> yuv420p (dither) -> yuv422p10le in one launch")
    s1 = ops.Scaler("yuv420p10le", 1280, 720, "yuv420p", 1920, 1080, flags="bicubic")
    s2 = ops.Scaler("yuv420p", 1920, 1080, "yuv422p10le", 1920, 1080, flags="bicubic")
    mid = FrameBatch("yuv420p", 1920, 1080, n, device=dev)
    ms = timed(lambda: (s1(c720, mid), s2(mid, c1080)))
    report("chain_two_launch_720p10_to_1080p422p10", "strip_kernel + scale_kernel", ms, plane_bytes(c720),
           plane_bytes(c1080), "round-1 path: yuv420p intermediate in HBM (its bytes not counted)")
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
