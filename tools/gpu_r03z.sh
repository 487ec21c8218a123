#!/bin/bash
# r03z: the down tasks read the L2L transfer matrices through the caches (build/ab_rg) vs staged in LDS
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03z
bash tools/gpu_ab_libs.sh r03z base rg rg base || exit 1
for n in base rg base rg; do
  if [ "$n" = base ]; then L=$PWD/aniso_amd/libaniso_mi355x.so; else L=$PWD/build/ab_$n/libaniso_mi355x.so; fi
  ANISO_LIB=$L timeout -k 10 200 python3 tools/shard_time.py 8 0 1 --native --no-timing > gpurun_out/r03z/w8_$n.log 2>&1 || { tail -20 gpurun_out/r03z/w8_$n.log; exit 1; }
  echo "$n w8 $(grep '^{' gpurun_out/r03z/w8_$n.log | cut -c1-90 | tr '\n' ' ')"
done
