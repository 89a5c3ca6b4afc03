#!/usr/bin/env python3
"""shares_summary.py -- slowest-rank prediction of the multi-GPU runs from tools/measure_shares.sh.

For an N-way split every rank renders its lattice share alone on one GPU; with one GPU per
rank the frame takes the slowest rank's time plus the gather.  Predicted N-GPU Mrays/s =
whole-frame rays / (max over ranks of the share's ms per frame + gather estimate); speed-up =
that / the whole frame's Mrays/s on one GPU.  The gather term is the measured fixed cost of one
RCCL gather at world size 1 plus the payload over one xGMI link (tools/gather_cost.py)."""
import argparse
import glob
import json
import os
import re

ap = argparse.ArgumentParser()
ap.add_argument("--dir", required=True)
ap.add_argument("--out", required=True)
ap.add_argument("--label", default="")
a = ap.parse_args()
J = lambda p: json.load(open(p))
gather = J(os.path.join(a.dir, "gather_cost.json")) if os.path.exists(os.path.join(a.dir, "gather_cost.json")) else {}
res = {"label": a.label, "rule": __doc__.split("\n\n")[1].replace("\n", " "), "workloads": {}}
for wl in ("head", "c5"):
    whole_p = os.path.join(a.dir, f"{wl}_whole.json")
    if not os.path.exists(whole_p):
        continue
    whole = J(whole_p)
    rays = whole["config"]["rays_per_step"]
    entry = {"whole_mrays": whole["value"], "whole_ms": whole["ms_per_step"], "splits": {}}
    for n in (2, 4, 8):
        files = sorted(glob.glob(os.path.join(a.dir, f"{wl}_{n}_*.json")), key=lambda p: int(re.findall(r"_(\d+)\.json$", p)[0]))
        if not files:
            continue
        ranks = [J(p) for p in files]
        ms = [r["ms_per_step"] for r in ranks]
        g = gather.get(f"{wl}_{n}way", {})
        # the collective's fixed cost (one torch.distributed.gather over RCCL at world size 1,
        # synchronised like bench.py's step) + the payload over one xGMI link (every peer
        # arrives over its own link, concurrently)
        g_ms = (g.get("gather_ms") or 0.0) + (g.get("xgmi_est_ms") or g.get("xgmi_estimate_ms") or 0.0)
        slow = max(ms)
        pred = rays / ((slow + g_ms) * 1e-3) / 1e6
        entry["splits"][n] = {
            "ranks": len(ranks), "per_rank_mrays": [r["value"] for r in ranks], "per_rank_ms": ms,
            "slowest_rank": ms.index(slow), "slowest_ms": slow, "fastest_ms": min(ms),
            "slowest_share_of_whole_rate": round(rays / n / (slow * 1e-3) / 1e6 / whole["value"], 4),
            "gather_ms_estimate": round(g_ms, 4),
            "predicted_mrays": round(pred, 1), "predicted_speedup": round(pred / whole["value"], 3),
        }
    res["workloads"][wl] = entry
res["gather"] = gather
json.dump(res, open(a.out, "w"), indent=1)
for wl, e in res["workloads"].items():
    for n, s in e["splits"].items():
        print(f"{wl} {n}-way: slowest rank {s['slowest_rank']} {s['slowest_ms']} ms, predicted {s['predicted_mrays']} "
              f"Mrays/s = {s['predicted_speedup']}x of {e['whole_mrays']}")
