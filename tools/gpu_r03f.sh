#!/bin/bash
# r03f: every rank's time at 8 shards (the max over ranks sets the step)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ranks_r03f.log
for r in 0 1 2 3 4 5 6 7; do
  timeout -k 10 120 python -u tools/ab_handles.py --world 8 --rank $r --reps 2 "" >> gpurun_out/ranks_r03f.log 2>&1 || { tail -20 gpurun_out/ranks_r03f.log; exit 1; }
done
grep "^{" gpurun_out/ranks_r03f.log
