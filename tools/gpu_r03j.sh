#!/bin/bash
# Timelines of the fused top-of-tree + M2L launch at 1 and 8 shards (tools/top_trace.py)
set -o pipefail
mkdir -p gpurun_out/r03j
export ANISO_TOP_TRACE=1
for a in "8 0" "8 1" "1 0"; do
  set -- $a
  timeout -k 10 200 python3 -u tools/top_trace.py $1 $2 gpurun_out/r03j/trace_w$1_r$2.npy >> gpurun_out/r03j/top_trace.log 2>&1 || { tail -20 gpurun_out/r03j/top_trace.log; exit 1; }
done
grep "^{" gpurun_out/r03j/top_trace.log
