"""Print the bench line summary and per-kernel averages of a tools/gpu_iter.sh run."""
import csv
import json
import sys

tag = sys.argv[1]
for line in open(f"gpurun_out/bench_{tag}.log"):
    if line.startswith("{"):
        d = json.loads(line)
        print(d["value"], d["ms_per_step"], d["stage_ms"], d["roofline"]["achieved"], d["roofline"]["frac"])
rows = list(csv.DictReader(open(f"gpurun_out/prof_{tag}/run_kernel_trace.csv")))
last = {}
for r in rows:
    last.setdefault(r["Kernel_Name"].split("(")[0], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for r in csv.DictReader(open(f"gpurun_out/prof_{tag}/run_kernel_stats.csv")):
    print(f"{r['Name'].split('(')[0][:40]:40s} {r['Calls']:>4s} {float(r['AverageNs'])/1e3:9.2f} us")
per = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Kernel_Name"].split("(")[0], r["Grid_Size_X"]) for r in rows[-12:]]
for p in per:
    print("   last:", p)
