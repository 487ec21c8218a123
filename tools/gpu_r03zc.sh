#!/bin/bash
# r03zc: the 3-wave cluster M2L with the target's x coordinates in 8 VGPRs again
# (build/ab_v1) against HEAD (base, the two-value form) and 7a52c9b (prev): parity
# subset on v1, then wall time alternating the three builds; rank 0 of 8 (loopback)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03zc
L1=$PWD/build/ab_v1/libaniso_mi355x.so
ANISO_LIB=$L1 timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "clusters_match or config3_size_matches or block_operator_matches or eight_shards or fused or knobs" --timeout 200 --timeout-method thread > gpurun_out/r03zc/tests_v1.log 2>&1 || { tail -30 gpurun_out/r03zc/tests_v1.log; exit 1; }
tail -1 gpurun_out/r03zc/tests_v1.log
for n in base v1 prev base v1 prev; do
  if [ "$n" = base ]; then L=$PWD/aniso_amd/libaniso_mi355x.so; else L=$PWD/build/ab_$n/libaniso_mi355x.so; fi
  ANISO_LIB=$L timeout -k 10 200 python -u tools/ab_timing.py 60 > gpurun_out/r03zc/abt_$n.log 2>&1 || { tail -20 gpurun_out/r03zc/abt_$n.log; exit 1; }
  echo "$n $(grep '^{' gpurun_out/r03zc/abt_$n.log)"
done
for n in base v1 base v1; do
  if [ "$n" = base ]; then L=$PWD/aniso_amd/libaniso_mi355x.so; else L=$PWD/build/ab_$n/libaniso_mi355x.so; fi
  ANISO_LIB=$L timeout -k 10 200 python3 tools/shard_time.py 8 0 1 --native --no-timing > gpurun_out/r03zc/w8_$n.log 2>&1 || { tail -20 gpurun_out/r03zc/w8_$n.log; exit 1; }
  echo "$n w8 $(grep '^{' gpurun_out/r03zc/w8_$n.log | cut -c1-90 | tr '\n' ' ')"
done
