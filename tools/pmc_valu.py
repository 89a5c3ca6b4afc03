#!/usr/bin/env python3
"""pmc_valu.py -- VALU issue rate and lane utilisation of one kernel from a rocprofv3 --pmc pass.

Usage: pmc_valu.py --dir DIR [--kernel REGEX] --out profiles/x.json

DIR is the -d directory of `rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU
SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE`.  Per dispatch (launches shorter than 50 us --
the empty last step -- are left out):
  VALU issue fraction = SQ_INSTS_VALU / (CUs x cycles): a CU issues at most one wave64 VALU
      instruction per cycle (measured: tools/ubench_valu.hip saturates at 0.84-0.90 per
      CU-cycle for v_fma / v_max3 / v_perm / v_pk_fma); cycles = GRBM_GUI_ACTIVE / XCDs
  lane utilisation   = SQ_THREAD_CYCLES_VALU / (64 x SQ_INSTS_VALU)
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re

N_CU, N_XCD, VALU_PER_CU_CYCLE = 256, 8, 1


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--kernel", default=r"trace_refill_kernel<false")
    ap.add_argument("--out", required=True)
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    disp: dict[tuple, dict] = {}
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if not re.search(a.kernel, row.get("Kernel_Name", "")):
                    continue
                key = (f, row.get("Dispatch_Id", ""))
                d = disp.setdefault(key, {"ns": int(row["End_Timestamp"]) - int(row["Start_Timestamp"])})
                d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    ds = [d for d in disp.values() if d["ns"] > 50_000 and "SQ_INSTS_VALU" in d]
    if not ds:
        raise SystemExit(f"kernel {a.kernel!r}: no dispatches with counters under {a.dir}")
    tot = {k: sum(d.get(k, 0.0) for d in ds) for k in ("ns", "SQ_INSTS_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_INSTS_SALU",
                                                        "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "GRBM_GUI_ACTIVE")}
    cycles = tot["GRBM_GUI_ACTIVE"] / N_XCD
    res = {
        "kernel": a.kernel,
        "label": a.label,
        "dispatches": len(ds),
        "clock_ghz": round(cycles / tot["ns"], 3),
        "valu_issue_frac": round(tot["SQ_INSTS_VALU"] / (N_CU * VALU_PER_CU_CYCLE * cycles), 4),
        "valu_wave_instr_per_cu_cycle": round(tot["SQ_INSTS_VALU"] / (N_CU * cycles), 4),
        "lane_utilisation": round(tot["SQ_THREAD_CYCLES_VALU"] / (64.0 * tot["SQ_INSTS_VALU"]), 4),
        "valu_g_wave_instr_per_s": round(tot["SQ_INSTS_VALU"] / tot["ns"], 2),
        "salu_per_valu": round(tot["SQ_INSTS_SALU"] / tot["SQ_INSTS_VALU"], 3),
        "vmem_rd_per_valu": round(tot["SQ_INSTS_VMEM_RD"] / tot["SQ_INSTS_VALU"], 4),
        "lds_per_valu": round(tot["SQ_INSTS_LDS"] / tot["SQ_INSTS_VALU"], 4),
        "per_dispatch_valu_issue_frac": [round(d["SQ_INSTS_VALU"] / (N_CU * VALU_PER_CU_CYCLE * d["GRBM_GUI_ACTIVE"] / N_XCD), 3)
                                         for d in ds],
        "definition": "valu_issue_frac = wave64 VALU instructions / (256 CUs x cycles x VALU_PER_CU_CYCLE) with "
                      "VALU_PER_CU_CYCLE = %g (the fp32 single-opcode rate, tools/ubench_valu.hip); bench.py prices "
                      "the roofline against the highest counter-measured mixed-stream rate instead (1.73, "
                      "profiles/*_ubench_valu_pmc.json) and the spec 2; valu_wave_instr_per_cu_cycle is the raw "
                      "rate; lane utilisation = SQ_THREAD_CYCLES_VALU / (64 x SQ_INSTS_VALU)" % VALU_PER_CU_CYCLE,
    }
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
