#!/usr/bin/env python3
"""pmc_ubench.py -- counter-measured VALU issue rate of tools/ubench_valu.hip.

Usage: pmc_ubench.py --dir DIR --out profiles/x.json

DIR is the -d directory of
  rocprofv3 --pmc SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- tools/bin/ubench_valu
Per dispatch of spin<KIND> (each kind runs at 1, 2, 4, 8 waves per SIMD, every shape twice:
an untimed warm-up and the timed launch; both are kept):
  wave64 VALU instructions per CU-cycle = SQ_INSTS_VALU / (256 CUs x GRBM_GUI_ACTIVE / 8 XCDs)
  clock                                = GRBM_GUI_ACTIVE / 8 / duration
SQ_INSTS_VALU counts what the compiler emitted and the SQ issued, so the rate holds whatever
the source-level count of tools/ubench_valu.hip says.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re

N_CU, N_XCD = 256, 8
KINDS = {0: "v_fma_f32", 2: "v_max3_f32", 3: "v_perm_b32", 4: "add_u32+cvt_f32_ubyte+add_f32", 5: "v_pk_fma_f32",
         6: "v_mul_lo_u32+v_add"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    disp: dict[tuple, dict] = {}
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                m = re.search(r"spin<(\d+)>", row.get("Kernel_Name", ""))
                if not m:
                    continue
                key = (f, row.get("Dispatch_Id", ""))
                d = disp.setdefault(key, {"kind": int(m.group(1)), "grid": int(row.get("Grid_Size", 0) or 0),
                                          "ns": int(row["End_Timestamp"]) - int(row["Start_Timestamp"]),
                                          "id": int(row.get("Dispatch_Id", 0) or 0)})
                d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    rows = []
    for d in sorted(disp.values(), key=lambda d: d["id"]):
        cyc = d.get("GRBM_GUI_ACTIVE", 0.0) / N_XCD
        if cyc <= 0 or "SQ_INSTS_VALU" not in d:
            continue
        waves_per_simd = d["grid"] // (256 * N_CU) if d["grid"] else None
        rows.append({"kind": KINDS.get(d["kind"], str(d["kind"])), "waves_per_simd": waves_per_simd,
                     "ms": round(d["ns"] / 1e6, 3), "clock_ghz": round(cyc / d["ns"], 3),
                     "valu_wave_instr_per_cu_cycle": round(d["SQ_INSTS_VALU"] / (N_CU * cyc), 3),
                     "sq_busy_frac": round(d.get("SQ_BUSY_CYCLES", 0.0) / max(d.get("GRBM_GUI_ACTIVE", 1.0), 1.0), 3)})
    best = max((r["valu_wave_instr_per_cu_cycle"] for r in rows), default=None)
    res = {"label": a.label, "counters": "SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE", "dispatches": rows,
           "max_valu_wave_instr_per_cu_cycle": best}
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    for r in rows:
        print(f"{r['kind']:30s} waves/SIMD {r['waves_per_simd']}: {r['valu_wave_instr_per_cu_cycle']:.3f} "
              f"wave64 VALU instr per CU-cycle at {r['clock_ghz']:.2f} GHz ({r['ms']:.3f} ms)")
    print("max", best)


if __name__ == "__main__":
    main()
