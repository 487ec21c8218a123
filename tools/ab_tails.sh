# rank-of-8 schedule (loopback, no stage events) with the partial tasks as tails of the
# bottom tier (default) against the pack launch (ANISO_UP_TAILS=0), separate processes
# interleaved; then a kernel trace of rank 0 with the tails.  usage: bash tools/ab_tails.sh TAG
set -o pipefail
T=${1:-r06e}
mkdir -p gpurun_out/$T
for rep in 1 2 3; do
  for v in 1 0; do
    echo "## ANISO_UP_TAILS=$v rep $rep"
    ANISO_UP_TAILS=$v timeout -k 10 200 python -u tools/shard_time.py 8 0 3 5 --native --no-timing || exit 1
  done
done > gpurun_out/$T/ab.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/tr -o run -- python3 tools/shard_time.py 8 0 --native --no-timing > gpurun_out/$T/trace_run.log 2>&1 || exit 1
python3 tools/trace_last.py $(find gpurun_out/$T/tr -name "*kernel_trace.csv" | head -1) > gpurun_out/$T/last.txt
