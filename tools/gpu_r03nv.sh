#!/bin/bash
# r03nv: near field as the last blocks of the fused launch (ANISO_NEAR_IN_TOP=1) on a
# rank of 8 (phase 2) and at 1 GPU: parity with the knob on, A/B, timelines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03nv
ANISO_NEAR_IN_TOP=1 timeout -k 10 400 python -u -m pytest tests/ -x -q --timeout 300 --timeout-method thread -m gpu -k "block_operator or clusters_match or fused or shard or phase or config3" > gpurun_out/r03nv/tests_on.log 2>&1 || { tail -40 gpurun_out/r03nv/tests_on.log; exit 1; }
tail -1 gpurun_out/r03nv/tests_on.log
timeout -k 10 300 python -u tools/ab_handles.py --world 8 --reps 4 "" "ANISO_NEAR_IN_TOP=1" > gpurun_out/r03nv/ab_w8.log 2>&1 || { tail -20 gpurun_out/r03nv/ab_w8.log; exit 1; }
grep "^{" gpurun_out/r03nv/ab_w8.log | cut -c1-330
for e in 0 1; do
  ANISO_NEAR_IN_TOP=$e timeout -k 10 200 python3 tools/shard_time.py 8 0 1 --native --no-timing > gpurun_out/r03nv/w8_$e.log 2>&1 || { tail -20 gpurun_out/r03nv/w8_$e.log; exit 1; }
  echo "near_in_top $e $(grep '^{' gpurun_out/r03nv/w8_$e.log | cut -c1-90 | tr '\n' ' ')"
  ANISO_NEAR_IN_TOP=$e ANISO_TOP_TRACE=1 timeout -k 10 200 python3 tools/top_trace.py 8 0 gpurun_out/r03nv/trace_w8_n$e.npy --native > gpurun_out/r03nv/trace_w8_n$e.log 2>&1 || { tail -20 gpurun_out/r03nv/trace_w8_n$e.log; exit 1; }
done
