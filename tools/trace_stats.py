#!/usr/bin/env python3
"""Per-kernel launch statistics from a rocprofv3 kernel trace (run_kernel_trace.csv),
over the TIMED launches only: the first `skip` launches of each kernel (the
bench's warm-up steps, which include first-touch of fresh output batches) are
dropped, so the mean is comparable with bench.py's HIP-event avg_launch_ms.

  python3 tools/trace_stats.py <run_kernel_trace.csv> <skip> [substring ...] > stats.csv
  PIXPATH_TRACE_BY_GRID=1: launches of one kernel with different grid sizes
  apart (e.g. the chain plan's luma and chroma launches of one instance)
"""
import os
import csv
import statistics
import sys
from collections import defaultdict


def main():
    path, skip = sys.argv[1], int(sys.argv[2])
    want = sys.argv[3:]
    d = defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if want and not any(w in name for w in want):
            continue
        if os.environ.get("PIXPATH_TRACE_BY_GRID"):
            g = [r[k] for k in sorted(r) if k.startswith("Grid_Size")]
            name = name.split("(")[0] + " grid=" + "x".join(g)
        d[name].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    print("kernel,launches_total,launches_timed,mean_ms,median_ms,min_ms,max_ms,stdev_ms,warmup_mean_ms")
    for name, ev in sorted(d.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
        ev.sort()
        dur = [(e - s) / 1e6 for s, e in ev]
        timed, warm = dur[skip:], dur[:skip]
        if not timed:
            continue
        short = name.split("(")[0].replace(",", ";")[:120]
        print("%s,%d,%d,%.4f,%.4f,%.4f,%.4f,%.4f,%s" % (
            short, len(dur), len(timed), statistics.mean(timed), statistics.median(timed), min(timed), max(timed),
            statistics.pstdev(timed), "%.4f" % statistics.mean(warm) if warm else ""))


if __name__ == "__main__":
    main()
