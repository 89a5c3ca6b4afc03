#!/usr/bin/env python3
"""pmc_summary.py DIR [DIR...] -- per-kernel average of every counter in rocprofv3 --pmc output."""
import collections
import csv
import glob
import os
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for root in sys.argv[1:]:
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(float)
        for row in csv.DictReader(open(f, newline="")):
            k = row["Kernel_Name"].replace("(anonymous namespace)::", "")[:48]
            per[(k, row.get("Dispatch_Id", ""), row["Counter_Name"])] += float(row["Counter_Value"])
        for (k, _, c), v in per.items():
            agg[k][c].append(v)
for k, d in sorted(agg.items()):
    if "rocclr" in k or "at::native" in k:
        continue
    print(k)
    for c, vs in sorted(d.items()):
        print(f"    {c:40s} {sum(vs) / len(vs):14.4g}  (n={len(vs)})")
