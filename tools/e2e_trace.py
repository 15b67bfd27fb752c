"""Summarise a rocprofv3 --kernel-trace --memory-copy-trace of the e2e_avpvs
leg (tools/gpu_e2e_trace.sh): per 20-ms bucket of the last second of the
trace, the busy time of each kernel family and copy direction."""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
ev = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("pp::", "")
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", "?")))
for f in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        kind = r.get("Direction") or r.get("Operation") or "copy"
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + kind, r.get("Queue_Id", "-")))
ev.sort()
end = max(e[1] for e in ev)
span = float(sys.argv[2]) if len(sys.argv) > 2 else 1.6
t0 = end - int(span * 1e9)
B = 20_000_000
busy = defaultdict(lambda: defaultdict(int))
for s, e, n, q in ev:
    if e < t0:
        continue
    s = max(s, t0)
    b = (s - t0) // B
    while s < e:
        be = t0 + (b + 1) * B
        busy[b][n] += min(e, be) - s
        s = min(e, be)
        b += 1
names = sorted({n for s, e, n, q in ev if e >= t0})
print("bucket_ms " + " ".join("%s" % n[:18] for n in names))
for b in sorted(busy):
    print("%6d    " % (b * 20) + " ".join("%18.1f" % (busy[b][n] / 1e6) for n in names))
qs = defaultdict(set)
for s, e, n, q in ev:
    if e >= t0:
        qs[n].add(q)
print("queues:", {n: sorted(v) for n, v in qs.items()})
