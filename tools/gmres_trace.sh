# kernel timeline of the bench's GMRES leg (restart 30 at 1M points): rocprofv3 kernel
# trace of a bench run with only that leg, then the kernels between two consecutive
# k_arn_column launches (one Arnoldi step + its look-ahead matvec).  usage: TAG
set -o pipefail
T=${1:-r06i}
mkdir -p gpurun_out/$T
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/tr -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --config2 0 --config5 0 --config4-sz 0 --no-solve --gmres 30 --warmup 5 > gpurun_out/$T/bench.log 2>&1 || exit 1
python3 - gpurun_out/$T $(find gpurun_out/$T/tr -name "*kernel_trace.csv" | head -1) <<'PY' > gpurun_out/$T/gmres_step.txt
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
col = [i for i, r in enumerate(rows) if "k_arn_column" in r["Kernel_Name"]]
for a, b in ((col[-12], col[-11]), (col[-6], col[-5])):
    t0 = int(rows[a]["End_Timestamp"])
    print("---- step", b)
    for r in rows[a + 1:b + 1]:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        print("%8.1f %8.1f %7.1f  %-50s q=%s" % (s, e, e - s, r["Kernel_Name"][:50], r["Queue_Id"]))
PY
