"""One timed GMRES cycle of the bench's leg from a rocprofv3 kernel trace: wall span
from the cycle's k_arn_begin to its last kernel, busy time per kernel family, and the
largest idle gaps between kernels (host-side stalls show up there).  Development tool.
usage: gmres_cycle.py KERNEL_TRACE_CSV"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
begins = [i for i, r in enumerate(rows) if "k_arn_begin" in r["Kernel_Name"]]
a = begins[-2]  # the last complete cycle: from its begin to the next cycle's begin
b = begins[-1] if len(begins) > 1 else len(rows)
cyc = rows[a:b]
t0 = int(cyc[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in cyc)
fam = collections.Counter()
for r in cyc:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")
    n = n.split("<")[0]
    fam[n] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
gaps = []
for p, q in zip(cyc, cyc[1:]):
    g = int(q["Start_Timestamp"]) - int(p["End_Timestamp"])
    gaps.append((g, p["Kernel_Name"][:40], q["Kernel_Name"][:40]))
gaps.sort(reverse=True)
steps = sum(1 for r in cyc if "k_arn_column" in r["Kernel_Name"])
print(f"cycle kernels {len(cyc)}  steps {steps}  wall {(t1 - t0) / 1e3:.1f} us  busy {sum(fam.values()) / 1e3:.1f} us  "
      f"idle {sum(max(g[0], 0) for g in gaps) / 1e3:.1f} us")
for n, v in fam.most_common(20):
    print(f"  {v / 1e3:9.1f} us  {n}")
print("largest gaps (us):")
for g in gaps[:12]:
    print(f"  {g[0] / 1e3:8.1f}  {g[1]} -> {g[2]}")
