# rank-of-8 schedule (loopback, no stage events) under knob settings, separate
# processes interleaved (3 repetitions), then a kernel trace of rank 0 under the first
# setting.  usage: TAG=r06l bash tools/ab_rank8.sh "A=1" "A=0"
set -o pipefail
T=${TAG:-r06l}
mkdir -p gpurun_out/$T
for rep in 1 2 3; do
  for cfg in "$@"; do
    echo "## $cfg rep $rep"
    env $cfg timeout -k 10 200 python -u tools/shard_time.py 8 ${RANKS:-0 3 5} --native --no-timing || exit 1
  done
done > gpurun_out/$T/ab.log 2>&1 || exit 1
env $1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/tr -o run -- python3 tools/shard_time.py 8 0 --native --no-timing > gpurun_out/$T/trace_run.log 2>&1 || exit 1
python3 tools/trace_last.py $(find gpurun_out/$T/tr -name "*kernel_trace.csv" | head -1) > gpurun_out/$T/last.txt
python3 - gpurun_out/$T/ab.log <<'PY'
import json, sys, collections
cur, res = None, collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith("## "):
        cur = l[3:].rsplit(" rep", 1)[0]
    elif l.startswith("{"):
        d = json.loads(l)
        res[(cur, d["rank"])].append(d["ms_per_apply"])
for k, v in sorted(res.items()):
    print(k, v, "min", min(v))
PY
