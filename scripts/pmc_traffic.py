#!/usr/bin/env python3
"""Per-launch HBM-side traffic of one kernel family from rocprofv3 --pmc runs.

usage: pmc_traffic.py <fetch_dir> <write_dir> <kernel-substring> [out.json]
FETCH_SIZE is doubled (gfx950 tallies 128-B requests at 64 B for 16-B/lane
streams: MI355X_MICROARCH.md, HBM section); WRITE_SIZE is taken as is.
Both are KB in rocprofv3's derived-counter definition."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_dispatch(d, counter, kern):
    vals = defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if kern not in name or row.get("Counter_Name") != counter:
                    continue
                key = (f, row.get("Dispatch_Id", row.get("Correlation_Id", "")))
                vals[key] += float(row.get("Counter_Value", 0))
    return list(vals.values())


def main():
    fetch_dir, write_dir, kern = sys.argv[1:4]
    fe = per_dispatch(fetch_dir, "FETCH_SIZE", kern)
    wr = per_dispatch(write_dir, "WRITE_SIZE", kern)
    if not fe or not wr:
        print(json.dumps({"kernel": kern, "error": "no samples", "fetch": len(fe), "write": len(wr)}))
        return
    fetch_b = 2.0 * 1024 * sum(fe) / len(fe)
    write_b = 1024 * sum(wr) / len(wr)
    out = {"kernel": kern, "dispatches": [len(fe), len(wr)], "fetch_bytes_per_launch": fetch_b,
           "write_bytes_per_launch": write_b, "traffic_bytes_per_launch": fetch_b + write_b,
           "correction": "FETCH_SIZE x2 (gfx950 128-B requests tallied at 64 B); sizes in KB x 1024"}
    print(json.dumps(out))
    if len(sys.argv) > 4:
        json.dump(out, open(sys.argv[4], "w"), indent=1)


if __name__ == "__main__":
    main()
