#!/bin/bash
# r03zb: r03za's bench (708/s) vs r03v (752/s): HEAD vs the commit before the 128-VGPR
# near field (build/ab_prev = 7a52c9b's csrc), same box; in-process knob A/B; block
# solve wall time over repeated calls
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03zb
for n in base prev base prev; do
  if [ "$n" = base ]; then L=$PWD/aniso_amd/libaniso_mi355x.so; else L=$PWD/build/ab_$n/libaniso_mi355x.so; fi
  ANISO_LIB=$L timeout -k 10 200 python -u tools/ab_timing.py 60 > gpurun_out/r03zb/abt_$n.log 2>&1 || { tail -20 gpurun_out/r03zb/abt_$n.log; exit 1; }
  echo "$n $(grep '^{' gpurun_out/r03zb/abt_$n.log)"
done
timeout -k 10 400 python -u tools/ab_handles.py --reps 4 "" "ANISO_NEAR_WPE=3" "ANISO_OVERLAP=0" "ANISO_HM_WPE=8,ANISO_OVERLAP=0" "ANISO_HM_WPE=8,ANISO_NEAR_WPE=3" > gpurun_out/r03zb/ab_w1.log 2>&1 || { tail -20 gpurun_out/r03zb/ab_w1.log; exit 1; }
grep "^{" gpurun_out/r03zb/ab_w1.log | cut -c1-330
timeout -k 10 200 python -u tools/solve_repeat.py > gpurun_out/r03zb/solve.log 2>&1 || { tail -20 gpurun_out/r03zb/solve.log; exit 1; }
grep "^{" gpurun_out/r03zb/solve.log
