#!/usr/bin/env python3
"""Per-case HBM traffic of tools/aux_kernels.py from two rocprofv3 PMC passes.

Usage: aux_pmc.py FETCH_CSV WRITE_CSV AUX_JSON LAUNCHES OUT_JSON

aux_kernels.py runs its cases in a fixed order, each as 1 warm-up + LAUNCHES
timed calls; a call is one dispatch, except stall_compose (one dispatch per
256 output frames).  The pp:: dispatches of each pass are assigned to the cases
in that order and averaged per call.  Read bytes = 2 x FETCH_SIZE (gfx950,
MI355X_MICROARCH.md HBM section); FETCH_SIZE / WRITE_SIZE are KiB.
"""
import csv
import json
import sys


def dispatches(path, counter):
    rows = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or "pp::" not in r["Kernel_Name"]:
            continue
        d = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(rows))
        rows[d] = rows.get(d, 0.0) + float(r["Counter_Value"]) * 1024.0
    return [rows[k] for k in sorted(rows)]


def main():
    fetch_csv, write_csv, aux_json, launches, out = sys.argv[1:6]
    launches = int(launches)
    cases = json.load(open(aux_json))
    fetch, write = dispatches(fetch_csv, "FETCH_SIZE"), dispatches(write_csv, "WRITE_SIZE")
    res, i = [], 0
    for c in cases:
        per_call = -(-c["frames"] // 256) if c["kernel"].startswith("stall") else 1
        n = (1 + launches) * per_call
        f, w = fetch[i:i + n], write[i:i + n]
        i += n
        calls = 1 + launches
        rd, wr = 2.0 * sum(f) / calls, sum(w) / calls
        alg = c["bytes_read"] + c["bytes_written"]
        res.append({"case": c["case"], "kernel": c["kernel"], "hbm_read": rd, "hbm_write": wr,
                    "hbm_bytes_per_call": rd + wr, "algorithmic_bytes": alg,
                    "traffic_over_algorithmic": round((rd + wr) / alg, 4)})
    if i != len(fetch) or i != len(write):
        res.append({"warning": "dispatch count mismatch: used %d, fetch %d, write %d" % (i, len(fetch), len(write))})
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
