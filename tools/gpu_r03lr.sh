#!/bin/bash
# r03lr: the one-block cluster M2L at 4 waves per SIMD (<= 128 VGPRs, m2l_hc_cluster<LR>):
# 4-wave workgroups where LDS allows 4 per CU (shards), 8-wave ones (2 per CU) for
# 64-target clusters; the near field at 128 VGPRs.  Parity, then same-process A/B
# at 1 GPU and a rank of 8, fused top launch and (variant build) separate tiers.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03lr
timeout -k 10 500 python -u -m pytest tests/ -x -q --timeout 300 --timeout-method thread -m gpu -k "block_operator or clusters_match or fused or shard or phase or config3 or knob" > gpurun_out/r03lr/tests.log 2>&1 || { tail -40 gpurun_out/r03lr/tests.log; exit 1; }
tail -1 gpurun_out/r03lr/tests.log
timeout -k 10 400 python -u tools/ab_handles.py --reps 4 "ANISO_HM_WPE=3" "ANISO_HM_WPE=8" "ANISO_NEAR_WPE=4" "ANISO_HM_WPE=8,ANISO_NEAR_WPE=4" > gpurun_out/r03lr/ab_w1.log 2>&1 || { tail -20 gpurun_out/r03lr/ab_w1.log; exit 1; }
grep "^{" gpurun_out/r03lr/ab_w1.log | cut -c1-260
ANISO_LIB=$PWD/build/ab_nofused/libaniso_mi355x.so timeout -k 10 400 python -u tools/ab_handles.py --reps 3 "ANISO_HM_WPE=3" "ANISO_HM_WPE=8" "ANISO_HM_WPE=8,ANISO_NEAR_WPE=4" > gpurun_out/r03lr/ab_w1_nofused.log 2>&1 || { tail -20 gpurun_out/r03lr/ab_w1_nofused.log; exit 1; }
grep "^{" gpurun_out/r03lr/ab_w1_nofused.log | cut -c1-260
timeout -k 10 300 python -u tools/ab_handles.py --world 8 --reps 4 "ANISO_HM_WPE=3" "" "ANISO_NEAR_WPE=4" > gpurun_out/r03lr/ab_w8.log 2>&1 || { tail -20 gpurun_out/r03lr/ab_w8.log; exit 1; }
grep "^{" gpurun_out/r03lr/ab_w8.log | cut -c1-260
ANISO_LIB=$PWD/build/ab_nofused/libaniso_mi355x.so timeout -k 10 300 python -u tools/ab_handles.py --world 8 --reps 4 "ANISO_HM_WPE=3" "" > gpurun_out/r03lr/ab_w8_nofused.log 2>&1 || { tail -20 gpurun_out/r03lr/ab_w8_nofused.log; exit 1; }
grep "^{" gpurun_out/r03lr/ab_w8_nofused.log | cut -c1-260
for e in 3 0; do
  ANISO_HM_WPE=$e timeout -k 10 200 python3 tools/shard_time.py 8 0 1 --native --no-timing > gpurun_out/r03lr/w8_$e.log 2>&1 || { tail -20 gpurun_out/r03lr/w8_$e.log; exit 1; }
  echo "wpe $e $(grep '^{' gpurun_out/r03lr/w8_$e.log | cut -c1-90 | tr '\n' ' ')"
done
