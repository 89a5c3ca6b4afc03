#!/usr/bin/env python3
"""pmc_traffic.py -- per-launch HBM bytes of one kernel from rocprofv3 --pmc passes.

Usage: pmc_traffic.py --fetch DIR --write DIR --kernel trace_kernel --out profiles/x.json

DIR is the -d directory of a `rocprofv3 --pmc FETCH_SIZE` (resp. WRITE_SIZE) run; every
*counter_collection.csv below it is read.  Corrections (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE counts 64 B per 128-B memory-side read request on gfx950, so it is doubled;
WRITE_SIZE is taken as is.  Both counters are in KB (rocprofv3 derived counters).
The two counters need separate passes (TCC slots: FETCH_SIZE 3, WRITE_SIZE 2 of 4).
Dispatches shorter than 50 us (the empty launch that ends a frame) are left out.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re


def per_dispatch(root: str, counter: str, kernel: str, min_ns: int = 50_000) -> list[float]:
    vals: dict[tuple[str, str], float] = {}
    files = glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {root}")
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter or not re.search(kernel, row.get("Kernel_Name", "")):
                    continue
                # the frame's last launch finds no query and returns at once: not a traversal step
                if "End_Timestamp" in row and int(row["End_Timestamp"]) - int(row["Start_Timestamp"]) < min_ns:
                    continue
                key = (f, row.get("Dispatch_Id", row.get("Correlation_Id", "")))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    # regex on the mangled name; the default excludes the instrumented (kCount=true) variant
    ap.add_argument("--kernel", default=r"trace_(refill_)?kernel(ILb0E|<false)")
    ap.add_argument("--out", required=True)
    ap.add_argument("--label", default="")
    # frames per traversal launch in the profiled run (bench.py --frames-per-call / its auto rule;
    # every profiled launch must render the same count): per-frame bytes for the bench line
    ap.add_argument("--frames", type=int, default=1)
    a = ap.parse_args()
    fe = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel)
    wr = per_dispatch(a.write, "WRITE_SIZE", a.kernel)
    if not fe or not wr:
        raise SystemExit(f"kernel {a.kernel!r} not found (fetch {len(fe)}, write {len(wr)} dispatches)")
    fetch_kb = sum(fe) / len(fe)
    write_kb = sum(wr) / len(wr)
    fetch_b = 2.0 * fetch_kb * 1024.0  # gfx950 FETCH_SIZE x2 correction
    write_b = write_kb * 1024.0
    res = {
        "kernel": a.kernel,
        "label": a.label,
        "dispatches_fetch_pass": len(fe),
        "dispatches_write_pass": len(wr),
        "fetch_size_kb_per_launch_raw": round(fetch_kb, 1),
        "write_size_kb_per_launch": round(write_kb, 1),
        "fetch_bytes_per_launch_corrected": round(fetch_b),
        "write_bytes_per_launch": round(write_b),
        "hbm_bytes_per_launch": round(fetch_b + write_b),
        "frames_per_launch": a.frames,
        "hbm_bytes_per_frame": round((fetch_b + write_b) / max(1, a.frames)),
        "write_bytes_per_frame": round(write_b / max(1, a.frames)),
        "correction": "FETCH_SIZE x2 (gfx950 tallies 128-B read requests at 64 B); WRITE_SIZE as is",
    }
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
