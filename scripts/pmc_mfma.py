#!/usr/bin/env python3
"""Counter-based MFMA utilisation of kernel families from one rocprofv3 --pmc run.

usage: pmc_mfma.py <pmc_dir> <out.json> <cus> name=substring[@resident_cus] ...

The run collects SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES and GRBM_GUI_ACTIVE
(one pass: 2 SQ + 1 GRBM counters) with --kernel-trace.  Per dispatch:
  kernel cycles  = GRBM_GUI_ACTIVE / 8   (summed over the 8 XCDs;
                   MI355X_MICROARCH.md "DVFS give-back")
  chip share     = SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x cus x kernel cycles)
  implied MFMAs  = SQ_VALU_MFMA_BUSY_CYCLES / 16 (v_mfma_f32_16x16x32_{f16,bf16}
                   hold a SIMD's matrix pipe 16 cycles: the guide's constants table)
The chip share is the counter analogue of the bench line's algorithmic
fraction: a persistent recurrence on 128 of 256 CUs can reach at most 0.5 of
it; `per_resident_cu` divides by the CUs the kernel's workgroups hold instead
(`@resident_cus` on the command line: the pinned recurrences launch 256
workgroups of which only dirs x groups x 32 stay, one per CU).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def rows(d, pattern):
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                yield f, r


def main():
    pmc_dir, out_path, cus = sys.argv[1], sys.argv[2], int(sys.argv[3])
    fams, res = {}, {}
    for a in sys.argv[4:]:
        name, sub = a.split("=", 1)
        sub, _, r = sub.partition("@")
        fams[name] = sub
        if r:
            res[name] = int(r)
    per = defaultdict(lambda: defaultdict(dict))  # family -> dispatch -> counter -> value
    for f, r in rows(pmc_dir, "*counter_collection*.csv"):
        name = r.get("Kernel_Name", "")
        for fam, sub in fams.items():
            if sub in name:
                key = (f, r.get("Dispatch_Id", r.get("Correlation_Id", "")))
                c = r.get("Counter_Name")
                per[fam][key][c] = per[fam][key].get(c, 0.0) + float(r.get("Counter_Value", 0))
    dur = defaultdict(list)
    for f, r in rows(pmc_dir, "*kernel_trace*.csv"):
        name = r.get("Kernel_Name", "")
        for fam, sub in fams.items():
            if sub in name:
                try:
                    dur[fam].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
                except (KeyError, ValueError):
                    pass
    out = {"counters": "SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE (one --pmc pass)",
           "formula": "MFMA busy / (4 SIMDs x CUs x GRBM_GUI_ACTIVE/8)", "cus": cus}
    for fam, disp in per.items():
        vals = [v for v in disp.values() if "SQ_VALU_MFMA_BUSY_CYCLES" in v and v.get("GRBM_GUI_ACTIVE")]
        if not vals:
            out[fam] = {"error": "no samples"}
            continue
        busy = sum(v["SQ_VALU_MFMA_BUSY_CYCLES"] for v in vals) / len(vals)
        kc = sum(v["GRBM_GUI_ACTIVE"] for v in vals) / len(vals) / 8.0
        resident = res.get(fam)
        e = {"dispatches": len(vals), "mfma_busy_cycles_per_launch": busy, "kernel_cycles_per_launch": kc,
             "implied_mfma_16cyc_per_launch": busy / 16.0, "chip_share": busy / (4.0 * cus * kc)}
        if resident:
            e["resident_cus"] = resident
            e["per_resident_cu"] = busy / (4.0 * resident * kc)
        if dur.get(fam):
            ns = sum(dur[fam]) / len(dur[fam])
            e["avg_duration_ms"] = ns / 1e6
            e["effective_clock_ghz"] = kc / ns
        out[fam] = e
    print(json.dumps(out, indent=1))
    with open(out_path, "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
