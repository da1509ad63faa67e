#!/usr/bin/env python3
"""Critical-path view of the last training step in a rocprofv3 kernel trace:
kernels in start order with queue, start/end (us from the step start) and
the idle gaps of the compute queue.  usage: timeline.py run_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
fw = [i for i, r in enumerate(rows) if "rnn_fwd_rec6" in r["Kernel_Name"]]
i0 = fw[-5]
while i0 > 0 and "clip_sgd" not in rows[i0 - 1]["Kernel_Name"]:
    i0 -= 1
seg = rows[i0:]
t0 = int(seg[0]["Start_Timestamp"])
rec_q = next(r["Queue_Id"] for r in seg if "rnn_fwd_rec6" in r["Kernel_Name"])
busy_end = None
idle = 0.0
for r in seg:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").replace("kctc::", "")
    name = name.split("(")[0][:58]
    gap = ""
    if r["Queue_Id"] == rec_q:
        if busy_end is not None and s > busy_end:
            idle += s - busy_end
            gap = f"  gap {s - busy_end:6.1f}"
        busy_end = max(busy_end or e, e)
    if len(sys.argv) < 3 or e - s > float(sys.argv[2]) or gap:
        print(f"q{r['Queue_Id']:>2} {s:10.1f} {e:10.1f} {e - s:9.1f}  {name}{gap}")
print(f"step span {(int(seg[-1]['End_Timestamp']) - t0) / 1e3:.1f} us, compute-queue idle {idle:.1f} us")
