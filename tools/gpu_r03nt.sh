#!/bin/bash
# r03nt: the near field as the last blocks of the fused top-of-tree + M2L launch
# (ANISO_NEAR_IN_TOP): parity subset, same-process A/B at 1 GPU, timelines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03nt
timeout -k 10 600 python -u -m pytest tests/ -x -q --timeout 300 --timeout-method thread -m gpu -k "block or harmonic or cluster or fused or near or top" > gpurun_out/r03nt/tests.log 2>&1 || { tail -40 gpurun_out/r03nt/tests.log; exit 1; }
tail -2 gpurun_out/r03nt/tests.log
timeout -k 10 300 python -u tools/ab_handles.py --reps 4 "ANISO_NEAR_IN_TOP=0" "" > gpurun_out/r03nt/ab_w1.log 2>&1 || { tail -20 gpurun_out/r03nt/ab_w1.log; exit 1; }
grep "^{" gpurun_out/r03nt/ab_w1.log | cut -c1-330
for e in 0 1; do
  ANISO_NEAR_IN_TOP=$e ANISO_TOP_TRACE=1 timeout -k 10 200 python3 tools/top_trace.py 1 0 gpurun_out/r03nt/trace_n$e.npy > gpurun_out/r03nt/trace_n$e.log 2>&1 || { tail -20 gpurun_out/r03nt/trace_n$e.log; exit 1; }
  echo "near_in_top $e $(grep '^{' gpurun_out/r03nt/trace_n$e.log | cut -c1-200)"
done
