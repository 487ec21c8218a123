#!/bin/bash
# r03y: the in-cluster partner products added by all 4 lanes of a quad (LDS atomics) vs
# reduced by DPP first (build/ab_qs: -DANISO_DUAL_QUADSUM); 1 GPU and one rank of 8
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03y
bash tools/gpu_ab_libs.sh r03y base sp sp base || exit 1
for n in base sp base sp; do
  if [ "$n" = base ]; then L=$PWD/aniso_amd/libaniso_mi355x.so; else L=$PWD/build/ab_$n/libaniso_mi355x.so; fi
  ANISO_LIB=$L timeout -k 10 200 python3 tools/shard_time.py 8 0 1 --native --no-timing > gpurun_out/r03y/w8_$n.log 2>&1 || { tail -20 gpurun_out/r03y/w8_$n.log; exit 1; }
  echo "$n w8 $(grep '^{' gpurun_out/r03y/w8_$n.log | cut -c1-90 | tr '\n' ' ')"
done
