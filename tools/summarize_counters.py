#!/usr/bin/env python3
"""Average every counter per kernel over the PMC passes in a directory (p*/run_counter_collection.csv)."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "pp::" not in k:
            continue
        k = k.split("(")[0].replace("void ", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        agg[k]["_VGPR"] = [float(r["VGPR_Count"])]
        agg[k]["_LDS"] = [float(r["LDS_Block_Size"])]
for k, cs in agg.items():
    print("==", k)
    for c in sorted(cs):
        v = cs[c]
        print("  %-28s %14.4g" % (c, sum(v) / len(v)))
