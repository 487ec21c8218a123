#!/bin/bash
# r03bb: cross-cluster pairs read once (partner products by global atomics): parity, timing, counters
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03bb
timeout -k 10 1000 python -u -m pytest tests/ -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r03bb/tests.log 2>&1 || { tail -40 gpurun_out/r03bb/tests.log; exit 1; }
tail -2 gpurun_out/r03bb/tests.log
timeout -k 10 300 python -u tools/ab_handles.py --reps 4 "ANISO_HM_XDUAL=0" "" > gpurun_out/r03bb/ab_w1.log 2>&1 || { tail -20 gpurun_out/r03bb/ab_w1.log; exit 1; }
grep "^{" gpurun_out/r03bb/ab_w1.log | cut -c1-330
for e in 0 1; do
  ANISO_HM_XDUAL=$e timeout -k 10 200 python3 tools/shard_time.py 8 0 1 --native --no-timing > gpurun_out/r03bb/w8_$e.log 2>&1 || { tail -20 gpurun_out/r03bb/w8_$e.log; exit 1; }
  echo "xdual $e $(grep '^{' gpurun_out/r03bb/w8_$e.log | cut -c1-90 | tr '\n' ' ')"
done
