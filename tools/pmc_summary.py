#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE CSVs per kernel (per launch).

MI355X_MICROARCH.md, HBM section: FETCH_SIZE and WRITE_SIZE are in KB; on gfx950
FETCH_SIZE reports exactly half the bytes of a wide coalesced streaming read, so it
is doubled here before being compared with algorithmic byte counts.
usage: pmc_summary.py <fetch_csv> <write_csv> <out_json>
"""
import collections
import csv
import json
import sys


def per_kernel(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}, {k: len(v) for k, v in agg.items()}


def main():
    fetch, launches = per_kernel(sys.argv[1], "FETCH_SIZE")
    write, _ = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {"note": "bytes per launch; fetch_bytes = 2 x FETCH_SIZE(KB) x 1024 (gfx950 correction), "
                   "write_bytes = WRITE_SIZE(KB) x 1024; traffic = fetch + write",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f = 2.0 * fetch.get(k, 0.0) * 1024.0
        w = write.get(k, 0.0) * 1024.0
        out["kernels"][k] = {"fetch_size_kb_raw": fetch.get(k), "write_size_kb_raw": write.get(k),
                             "fetch_bytes": f, "write_bytes": w, "traffic_bytes": f + w,
                             "launches": launches.get(k, 0)}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    for k, v in out["kernels"].items():
        print(f"{k:40s} traffic {v['traffic_bytes'] / 1e9:9.4f} GB")


if __name__ == "__main__":
    main()
