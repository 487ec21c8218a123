#!/bin/bash
# r03l: LDS-ring cluster M2L (lane-held pair indices) -- cluster parity, then depth A/B at 1 and 8 shards
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03l
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu \
  -k "clusters or knobs" > gpurun_out/r03l/tests.log 2>&1 || { tail -30 gpurun_out/r03l/tests.log; exit 1; }
tail -2 gpurun_out/r03l/tests.log
timeout -k 10 300 python -u tools/ab_handles.py "ANISO_HM_RING=0" "ANISO_HM_RING=2" "ANISO_HM_RING=3" "ANISO_HM_RING=4" > gpurun_out/r03l/ab_w1.log 2>&1 || { tail -20 gpurun_out/r03l/ab_w1.log; exit 1; }
grep "^{" gpurun_out/r03l/ab_w1.log | cut -c1-300
timeout -k 10 300 python -u tools/ab_handles.py --world 8 "ANISO_HM_RING=0" "ANISO_HM_RING=2" "ANISO_HM_RING=3" "ANISO_HM_RING=4" > gpurun_out/r03l/ab_w8.log 2>&1 || { tail -20 gpurun_out/r03l/ab_w8.log; exit 1; }
grep "^{" gpurun_out/r03l/ab_w8.log | cut -c1-300
