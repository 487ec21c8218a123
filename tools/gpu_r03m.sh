#!/bin/bash
# r03m: LDS-ring cluster M2L, target multipole in VGPRs or LDS -- parity, then A/B at 1 and 8 shards
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03m
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu \
  -k "clusters or knobs" > gpurun_out/r03m/tests.log 2>&1 || { tail -30 gpurun_out/r03m/tests.log; exit 1; }
tail -2 gpurun_out/r03m/tests.log
timeout -k 10 300 python -u tools/ab_handles.py "ANISO_HM_RING=0" "ANISO_HM_RING=3" "ANISO_HM_RING=3,ANISO_HM_RING_XL=1" "ANISO_HM_RING=2,ANISO_HM_RING_XL=1" "ANISO_HM_RING=3,ANISO_HM_RING_XL=1,ANISO_HM_CLDEPTH=2" "ANISO_HM_RING=2,ANISO_HM_RING_XL=1,ANISO_HM_CLDEPTH=2" > gpurun_out/r03m/ab_w1.log 2>&1 || { tail -20 gpurun_out/r03m/ab_w1.log; exit 1; }
grep "^{" gpurun_out/r03m/ab_w1.log | cut -c1-300
timeout -k 10 300 python -u tools/ab_handles.py --world 8 "ANISO_HM_RING=0" "ANISO_HM_RING=3" "ANISO_HM_RING=2" "ANISO_HM_RING=4" "ANISO_HM_RING=3,ANISO_HM_RING_XL=0" > gpurun_out/r03m/ab_w8.log 2>&1 || { tail -20 gpurun_out/r03m/ab_w8.log; exit 1; }
grep "^{" gpurun_out/r03m/ab_w8.log | cut -c1-300
