#!/usr/bin/env python3
"""Per-kernel averages (per launch) of every counter in one rocprofv3 --pmc CSV, plus
MfmaUtil = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) when
both are present (MI355X_MICROARCH.md: GRBM_GUI_ACTIVE is the sum over the 8 XCDs).
usage: counter_summary.py <counter_collection.csv> <out_json>"""
import collections
import csv
import json
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
out = {}
for k, c in agg.items():
    d = max(len(n[k]), 1)
    v = {name: val / d for name, val in c.items()}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in v and v.get("GRBM_GUI_ACTIVE"):
        v["mfma_util_pct"] = 100.0 * v["SQ_VALU_MFMA_BUSY_CYCLES"] / (v["GRBM_GUI_ACTIVE"] / 8.0 * 1024.0)
    if "SQ_INSTS_VALU_MFMA_MOPS_F32" in v:
        v["mfma_flop_f32"] = 512.0 * v["SQ_INSTS_VALU_MFMA_MOPS_F32"]
    v["dispatches"] = d
    out[k] = v
json.dump(out, open(sys.argv[2], "w"), indent=1)
for k, v in sorted(out.items()):
    if "k32" in k or "mfma_util_pct" in v:
        print(k[:40], {kk: round(vv, 3) for kk, vv in v.items() if kk in ("SQ_INSTS_VALU_MFMA_F32", "mfma_util_pct", "mfma_flop_f32", "GRBM_GUI_ACTIVE")})
