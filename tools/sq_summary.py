"""Per-kernel averages of the SQ counter passes of tools/sq_profile.sh."""
import csv
import glob
import sys
from collections import defaultdict

tag = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"gpurun_out/{tag if tag.startswith('l2_') else 'sq_' + tag}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in sorted(acc.items()):
    if "aniso" not in k:
        continue
    print(k)
    print("   " + "  ".join(f"{n}={sum(v) / len(v):.4g}" for n, v in sorted(c.items())))
