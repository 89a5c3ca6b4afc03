#!/usr/bin/env python3
"""timeline.py -- the last frame's kernels from a rocprofv3 --kernel-trace CSV (start, duration,
stream), to see how the logic / trace launches of the slot pipelines overlap.
Usage: timeline.py KT_DIR [n_last]"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "rocclr" not in r["Kernel_Name"]][-n:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    k = r["Kernel_Name"]
    name = "trace" if "trace" in k else "logic" if "logic" in k else k.split("(")[0][-24:]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{name:24s} q{r.get('Queue_Id', r.get('Stream_Id', '?')):>3s} start {(s - t0) / 1e6:8.3f}  end {(e - t0) / 1e6:8.3f}  dur {(e - s) / 1e6:7.3f}")
