#!/bin/bash
# r03o: raised priority of the fused launch's up blocks; ring policy -- parity, A/B at 1 and 8 shards, timeline
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu \
  -k "clusters or knobs or fused" > gpurun_out/r03o/tests.log 2>&1 || { tail -30 gpurun_out/r03o/tests.log; exit 1; }
tail -2 gpurun_out/r03o/tests.log
timeout -k 10 300 python -u tools/ab_handles.py "ANISO_TOP_PRIO=0" "" "ANISO_HM_RING=3" > gpurun_out/r03o/ab_w1.log 2>&1 || { tail -20 gpurun_out/r03o/ab_w1.log; exit 1; }
grep "^{" gpurun_out/r03o/ab_w1.log | cut -c1-300
timeout -k 10 300 python -u tools/ab_handles.py --world 8 "ANISO_TOP_PRIO=0" "" "ANISO_TOP_PRIO=0,ANISO_HM_RING=3" "ANISO_HM_RING=3" > gpurun_out/r03o/ab_w8.log 2>&1 || { tail -20 gpurun_out/r03o/ab_w8.log; exit 1; }
grep "^{" gpurun_out/r03o/ab_w8.log | cut -c1-300
ANISO_TOP_TRACE=1 timeout -k 10 200 python3 -u tools/top_trace.py 8 0 gpurun_out/r03o/trace_w8.npy > gpurun_out/r03o/trace_w8.log 2>&1 || { tail -20 gpurun_out/r03o/trace_w8.log; exit 1; }
grep "^{" gpurun_out/r03o/trace_w8.log | cut -c1-800
