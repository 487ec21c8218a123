"""Print the kernels of the last apply in a rocprofv3 kernel trace (times in us
from the first kernel after the previous down pass).  usage: trace_last.py CSV
[DOWN_KERNEL_PREFIX, default k_down_tier<5>: the block matvec's]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
key = sys.argv[2] if len(sys.argv) > 2 else "k_down_tier<5>"
idx = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
last, prev = idx[-1], idx[-2]
t0 = int(rows[prev + 1]["Start_Timestamp"])
for r in rows[prev + 1:last + 1]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    print("%8.1f %8.1f %7.1f  %-40s grid=%s q=%s" % (s, e, e - s, r["Kernel_Name"][:40], r["Grid_Size_X"], r["Queue_Id"]))
