#!/bin/bash
# r03n: launch timelines of the one-block and ring cluster forms at 8 and 1 shards
set -o pipefail
mkdir -p gpurun_out/r03n
export ANISO_TOP_TRACE=1
for cfg in "0 8" "3 8" "0 1" "3 1"; do
  set -- $cfg
  ANISO_HM_RING=$1 timeout -k 10 200 python3 -u tools/top_trace.py $2 0 gpurun_out/r03n/trace_ring$1_w$2.npy > gpurun_out/r03n/trace_ring$1_w$2.log 2>&1 || { tail -20 gpurun_out/r03n/trace_ring$1_w$2.log; exit 1; }
  echo "ring $1 world $2"; grep "^{" gpurun_out/r03n/trace_ring$1_w$2.log | cut -c1-1100
done
