#!/bin/bash
# Kernel trace of rank 0 of an N-way sharded block matvec (tools/shard_time.py) and
# the timeline of its last apply.  usage: tools/gpu_shardtrace.sh <tag> [world]
set -o pipefail
TAG=${1:-st}
W=${2:-8}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/shardtrace_$TAG -o run -- python3 tools/shard_time.py $W 0 > gpurun_out/shardtrace_$TAG.log 2>&1 || { tail -20 gpurun_out/shardtrace_$TAG.log; exit 1; }
grep "^{" gpurun_out/shardtrace_$TAG.log
python3 tools/trace_last.py gpurun_out/shardtrace_$TAG/run_kernel_trace.csv
