#!/bin/bash
# r03k: the LDS-ring cluster M2L -- parity of the cluster tests, then ring depth A/B at 1 and 8 shards
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03k
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu \
  -k "clusters or knobs or fused or deterministic or sz512 or eight_shards" > gpurun_out/r03k/tests.log 2>&1 || { tail -30 gpurun_out/r03k/tests.log; exit 1; }
tail -3 gpurun_out/r03k/tests.log
timeout -k 10 300 python -u tools/ab_handles.py "ANISO_HM_RING=0" "ANISO_HM_RING=2" "ANISO_HM_RING=3" "ANISO_HM_RING=4" > gpurun_out/r03k/ab_w1.log 2>&1 || { tail -20 gpurun_out/r03k/ab_w1.log; exit 1; }
grep "^{" gpurun_out/r03k/ab_w1.log | cut -c1-400
timeout -k 10 300 python -u tools/ab_handles.py --world 8 "ANISO_HM_RING=0" "ANISO_HM_RING=2" "ANISO_HM_RING=3" "ANISO_HM_RING=4" > gpurun_out/r03k/ab_w8.log 2>&1 || { tail -20 gpurun_out/r03k/ab_w8.log; exit 1; }
grep "^{" gpurun_out/r03k/ab_w8.log | cut -c1-400
ANISO_TOP_TRACE=1 timeout -k 10 200 python3 -u tools/top_trace.py 8 0 gpurun_out/r03k/trace_w8_r0.npy > gpurun_out/r03k/top_trace.log 2>&1 || { tail -20 gpurun_out/r03k/top_trace.log; exit 1; }
grep "^{" gpurun_out/r03k/top_trace.log | cut -c1-900
