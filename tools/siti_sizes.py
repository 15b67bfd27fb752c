"""SI/TI kernel time at 1080p and 2160p (600 frames, 10- and 8-bit) for the library PIXPATH_LIB points at
(HIP-event means over 5 calls after 1 warmup, torch's current stream). Measurement only."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "processing-chain_amd"))
from pixpath import ops  # noqa: E402

torch.manual_seed(0)
for (w, h, depth) in [(1920, 1080, 10), (3840, 2160, 10), (3840, 2160, 8)]:
    dt = torch.int16 if depth > 8 else torch.uint8
    hi = 1024 if depth > 8 else 256
    x = torch.randint(0, hi, (600, h, w), dtype=torch.int32, device="cuda").to(dt)
    ops.siti(x, depth)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        ops.siti(x, depth)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 5
    gbs = x.numel() * x.element_size() / (ms / 1e3) / 1e9
    print("%s %dx%d %d-bit %.4f ms %.0f GB/s" % (os.environ.get("PIXPATH_LIB", "current").split("/")[-1], w, h, depth, ms, gbs), flush=True)
    del x
    torch.cuda.empty_cache()
