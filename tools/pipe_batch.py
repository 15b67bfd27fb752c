"""pcie_pipeline rate against the pipeline batch size (measurement only)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "processing-chain_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
for b in [int(x) for x in sys.argv[1:]] or [30, 60, 120]:
    r = bench.pcie_pipeline(bench.WORKLOADS["config2"], 600, dev, batch=b)
    print(json.dumps({"batch": b, "frames_per_s": r["frames_per_s"], "pcie_gbs": r["pcie_gbs"]}), flush=True)
