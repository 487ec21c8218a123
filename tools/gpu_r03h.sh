#!/bin/bash
# r03h: config 4 (4M points, mode 0 forward operator) and 1M mode 0: one GPU vs every rank of 8
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/cfg4_r03h.log
for sz in 2048 1024; do
  timeout -k 10 200 python -u tools/ab_handles.py --ks 1 --sz $sz --reps 2 "" >> gpurun_out/cfg4_r03h.log 2>&1 || { tail -20 gpurun_out/cfg4_r03h.log; exit 1; }
  for r in 0 3 5 7; do
    timeout -k 10 200 python -u tools/ab_handles.py --ks 1 --sz $sz --world 8 --rank $r --reps 2 "" >> gpurun_out/cfg4_r03h.log 2>&1 || { tail -20 gpurun_out/cfg4_r03h.log; exit 1; }
  done
done
grep "^{" gpurun_out/cfg4_r03h.log | cut -c1-260
