#!/bin/bash
# r03ls: defaults after r03lr -- shards run the upper tiers as separate launches
# (ANISO_TOP_FUSED), the near field at 4 waves per SIMD (ANISO_NEAR_WPE): parity, A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03ls
timeout -k 10 600 python -u -m pytest tests/ -x -q --timeout 300 --timeout-method thread -m gpu -k "block_operator or clusters or fused or shard or phase or config3 or knob or near or solve" > gpurun_out/r03ls/tests.log 2>&1 || { tail -40 gpurun_out/r03ls/tests.log; exit 1; }
tail -1 gpurun_out/r03ls/tests.log
timeout -k 10 300 python -u tools/ab_handles.py --reps 4 "ANISO_NEAR_WPE=3" "" > gpurun_out/r03ls/ab_w1.log 2>&1 || { tail -20 gpurun_out/r03ls/ab_w1.log; exit 1; }
grep "^{" gpurun_out/r03ls/ab_w1.log | cut -c1-200
timeout -k 10 400 python -u tools/ab_handles.py --world 8 --reps 4 "ANISO_TOP_FUSED=1,ANISO_NEAR_WPE=3" "ANISO_TOP_FUSED=1" "ANISO_NEAR_WPE=3" "" > gpurun_out/r03ls/ab_w8.log 2>&1 || { tail -20 gpurun_out/r03ls/ab_w8.log; exit 1; }
grep "^{" gpurun_out/r03ls/ab_w8.log | cut -c1-260
for e in "ANISO_TOP_FUSED=1 ANISO_NEAR_WPE=3" "ANISO_TOP_FUSED=0 ANISO_NEAR_WPE=4"; do
  env $e timeout -k 10 200 python3 tools/shard_time.py 8 0 1 --native --no-timing > gpurun_out/r03ls/w8.log 2>&1 || { tail -20 gpurun_out/r03ls/w8.log; exit 1; }
  echo "$e $(grep '^{' gpurun_out/r03ls/w8.log | cut -c1-90 | tr '\n' ' ')"
done
