#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes into per-launch HBM traffic (profiles/pmc_traffic.json).

Usage: pmc_traffic.py FETCH_CSV WRITE_CSV KERNEL_TRACE_CSV OUT_JSON FRAMES_PER_LAUNCH

FETCH_SIZE / WRITE_SIZE are KiB (rocprofv3 derived counters).  Correction per
/opt/skills/guides/MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE
reports exactly half of the bytes of a wide coalesced streaming read, so the
read side is doubled; WRITE_SIZE is exact for 16-B/lane streaming stores
(other store widths are uncalibrated -- flagged in the output).
"""
import csv
import collections
import json
import os
import sys

# PIXPATH_TRACE_BY_GRID=1: launches of one kernel with different grid sizes
# apart (the chain plan's luma and chroma launches of one strip_kernel instance)
BY_GRID = bool(os.environ.get("PIXPATH_TRACE_BY_GRID"))


def _key(short, row):
    if not BY_GRID:
        return short
    g = 1
    for k, v in row.items():
        if k.startswith("Grid_Size") and v:
            g *= int(v)
    return "%s grid=%d" % (short, g)

KERNELS = {"scale_kernel": "pp::scale_kernel", "strip_kernel": "pp::strip_kernel", "siti_kernel": "pp::siti_kernel", "v210_kernel": "pp::v210_kernel",
           "pad_kernel": "pp::pad_kernel", "stall_kernel": "pp::stall_kernel", "cpvs_kernel": "pp::cpvs_kernel"}


def per_kernel(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        for short, pat in KERNELS.items():
            if pat in r["Kernel_Name"]:
                agg[_key(short, r)].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    fetch_csv, write_csv, trace_csv, out, frames = sys.argv[1:6]
    fetch = per_kernel(fetch_csv, "FETCH_SIZE")
    write = per_kernel(write_csv, "WRITE_SIZE")
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(trace_csv)):
        for short, pat in KERNELS.items():
            if pat in r["Kernel_Name"]:
                dur[_key(short, r)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    res = {"frames_per_launch": int(frames), "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes)",
           "correction": "read bytes = 2 x FETCH_SIZE (gfx950, MI355X_MICROARCH.md HBM section)", "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        rd = 2.0 * fetch.get(k, 0.0)
        wr = write.get(k, 0.0)
        res["kernels"][k] = {"fetch_size_bytes_raw": fetch.get(k), "read_bytes_corrected": rd, "write_bytes": wr,
                             "hbm_bytes_per_launch": rd + wr,
                             "avg_duration_ns": (sum(dur[k]) / len(dur[k])) if dur.get(k) else None}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
