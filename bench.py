#!/usr/bin/env python3
"""Benchmark of the MI355X raw-frame pixel path (BASELINE.json metric).

Workload (BASELINE.json configs[1], "config 2"): one 10 s 1080p60 SRC ->
  * P.910 SI/TI over 600 frames of 1920x1080 10-bit luma, and
  * 600 frames of 1280x720 yuv422p10le upscaled (lanczos, swscale-exact) to a
    1920x1080 yuv422p10le AVPVS.
A step = one pass of that hot path over the 600-frame batch, inputs resident in
HBM.  value = frames of that workload per second over all ranks (each frame
gets both its SI/TI and its AVPVS upscale).  Multi-GPU: one process per GPU,
each rank owns its own 600-frame PVS (PVS sharding, SURVEY.md section 8e, weak
scaling); the only collectives are the timing barrier and the max-over-ranks
of the elapsed time -- no data-path exchange.

Extra fields: roofline of the dominant kernel (the fused scaler) from HIP
events around its launches on the launch stream, the PMC traffic from a
separate rocprofv3 --pmc pass (profiles/, see tools/pmc_traffic.py), and the
CPU baseline (oracle/ C restatement, "port", bounded sample on host threads).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "processing-chain_amd"))

FRAMES = 600
SRC_W, SRC_H, DST_W, DST_H = 1280, 720, 1920, 1080
SCALE_BYTES_PER_FRAME = 3_686_400 + 8_294_400     # 720p + 1080p yuv422p10le
SITI_BYTES_PER_FRAME = 4_147_200                   # 1080p 10-bit luma, read once
HBM_PEAK_GBS = 8000.0                              # MI355X_MICROARCH.md: 8.0 TB/s spec
METRIC = "1080p yuv422p10 AVPVS frames/sec + SI/TI frames/sec; achieved HBM GB/s"
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=FRAMES)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-frames", type=int, default=4096,
                    help="upper bound on CPU-baseline frames (the sample also stops after --cpu-seconds)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    return ap.parse_args()


def cpu_baseline(args):
    """Oracle C restatement on host threads (ctypes releases the GIL)."""
    import threading
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po
    rng = np.random.default_rng(910)
    n = args.cpu_sample_frames
    nt = max(1, min(args.cpu_threads, n))
    src = [[rng.integers(64, 941, (SRC_H, SRC_W)).astype(np.uint16),
            rng.integers(64, 961, (SRC_H, SRC_W // 2)).astype(np.uint16),
            rng.integers(64, 961, (SRC_H, SRC_W // 2)).astype(np.uint16)] for _ in range(nt)]
    luma = [rng.integers(64, 941, (2, DST_H, DST_W)).astype(np.uint16) for _ in range(nt)]
    sws = [po.Sws(po.YUV422P10LE, SRC_W, SRC_H, po.YUV422P10LE, DST_W, DST_H, po.SWS_LANCZOS) for _ in range(nt)]

    done = [0] * nt

    def work(t):
        for i in range(t, n, nt):
            sws[t].scale(src[t])
            po.siti_c(luma[t], 10)  # 2 frames: SI of both, TI of the second
            done[t] += 1
            if time.perf_counter() - t0 > args.cpu_seconds:
                break
    t0 = time.perf_counter()
    th = [threading.Thread(target=work, args=(t,)) for t in range(nt)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t0
    n = sum(done)
    # each sample frame did one upscale and SI/TI of one frame (plus one extra SI)
    return {"value": n / dt, "unit": "frames/s", "cores": nt, "kind": "port",
            "sample": "%d frames, time-bounded at ~%gs (720p->1080p yuv422p10le lanczos + 1080p 10-bit SI/TI) on %d host threads, "
                      "oracle/pixoracle.c + siti_oracle.c (gcc -O2); ffmpeg is absent on the box" % (n, args.cpu_seconds, nt),
            "seconds": dt}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    from pixpath import ops
    from pixpath.frames import FrameBatch

    n = args.frames
    g = torch.Generator(device=dev)
    g.manual_seed(910 + rank)
    # synthetic inputs in the legal 10-bit range, generated in HBM
    src = FrameBatch("yuv422p10le", SRC_W, SRC_H, n, device=dev)
    for p, (lo, hi) in enumerate([(64, 941), (64, 961), (64, 961)]):
        v = src.view(p)
        v.copy_(torch.randint(lo, hi, v.shape, generator=g, device=dev, dtype=torch.int32).to(torch.uint16))
    dst = FrameBatch("yuv422p10le", DST_W, DST_H, n, device=dev)
    luma = torch.randint(64, 941, (n, DST_H, DST_W), generator=g, device=dev, dtype=torch.int32).to(torch.uint16)
    scaler = ops.Scaler("yuv422p10le", SRC_W, SRC_H, "yuv422p10le", DST_W, DST_H, flags="lanczos")
    torch.cuda.synchronize()

    ev = []

    def step(timed):
        if timed:
            a, b, c = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            a.record()
            scaler(src, dst)
            b.record()
            ops.siti(luma, 10)
            c.record()
            ev.append((a, b, c))
        else:
            scaler(src, dst)
            ops.siti(luma, 10)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    scale_ms = sum(a.elapsed_time(b) for a, b, _ in ev) / len(ev)
    siti_ms = sum(b.elapsed_time(c) for _, b, c in ev) / len(ev)
    ms_per_step = elapsed * 1000.0 / args.steps
    value = world * n * args.steps / elapsed

    if rank == 0:
        achieved = SCALE_BYTES_PER_FRAME * n / (scale_ms / 1000.0) / 1e9
        traffic = None
        if os.path.exists(PMC_FILE):
            try:
                pm = json.load(open(PMC_FILE))
                k = pm.get("kernels", {}).get("strip_kernel") or pm.get("kernels", {}).get("scale_kernel")
                if k and pm.get("frames_per_launch") == n:
                    traffic = k["hbm_bytes_per_launch"]
            except Exception:
                traffic = None
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u16",
            "data": "synthetic (seeded legal-range 10-bit noise, generated in HBM)",
            "config": {
                "workload": "config2: 10 s 1080p60 SRC -> SI/TI (1920x1080 10-bit luma) + 1280x720->1920x1080 "
                            "yuv422p10le lanczos AVPVS upscale",
                "frames_per_step_per_gpu": n,
                "parallelism": "pvs-sharded x%d (one process per GPU, no data-path collective)" % world,
            },
            "avpvs_fps_kernel": round(world * n / (scale_ms / 1000.0), 1),
            "siti_fps_kernel": round(world * n / (siti_ms / 1000.0), 1),
            "siti_achieved_gbs": round(SITI_BYTES_PER_FRAME * n / (siti_ms / 1000.0) / 1e9, 1),
            "roofline": {
                "bound": "hbm",
                "kernel": "strip_kernel (fused H+V polyphase over 256-column strips, one launch per 600-frame batch)",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "algorithmic_bytes_per_launch": SCALE_BYTES_PER_FRAME * n,
                "avg_launch_ms": round(scale_ms, 4),
            },
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(args)
            out["cpu_baseline"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in cb.items()}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
