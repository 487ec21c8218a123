#!/bin/bash
# r03dt: per-task phase timeline of the down pass (variant build with -DANISO_DOWN_TRACE)
set -o pipefail
export ANISO_LIB=$PWD/build/ab_dt/libaniso_mi355x.so
for w in 1 8; do
  timeout -k 10 200 python3 tools/down_trace.py $w 2>&1 | grep -v amdgpu.ids || exit 1
done
