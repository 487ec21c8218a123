#!/bin/bash
# r03nu: near groups interleaved with the clusters in the fused launch (ANISO_NEAR_TAIL)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03nu
timeout -k 10 300 python -u -m pytest tests/ -x -q --timeout 200 --timeout-method thread -m gpu -k "block_operator or clusters_match or fused" > gpurun_out/r03nu/tests.log 2>&1 || { tail -40 gpurun_out/r03nu/tests.log; exit 1; }
tail -1 gpurun_out/r03nu/tests.log
timeout -k 10 400 python -u tools/ab_handles.py --reps 4 "ANISO_NEAR_IN_TOP=0" "ANISO_NEAR_TAIL=100" "ANISO_NEAR_TAIL=60" "ANISO_NEAR_TAIL=30" "ANISO_NEAR_TAIL=0" > gpurun_out/r03nu/ab_w1.log 2>&1 || { tail -20 gpurun_out/r03nu/ab_w1.log; exit 1; }
grep "^{" gpurun_out/r03nu/ab_w1.log | cut -c1-200
for e in 60 30; do
  ANISO_NEAR_TAIL=$e ANISO_TOP_TRACE=1 timeout -k 10 200 python3 tools/top_trace.py 1 0 gpurun_out/r03nu/trace_t$e.npy > gpurun_out/r03nu/trace_t$e.log 2>&1 || { tail -20 gpurun_out/r03nu/trace_t$e.log; exit 1; }
done
