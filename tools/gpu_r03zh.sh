#!/bin/bash
# r03zh: the cluster M2L hands its targets to the waves through an LDS counter
# (build/ab_v5) instead of round-robin, against the in-tree build: parity subset on v5,
# wall time alternating; rank 0 of 8 (loopback)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03zh
L1=$PWD/build/ab_v5/libaniso_mi355x.so
ANISO_LIB=$L1 timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "clusters_match or config3_size_matches or block_operator_matches or eight_shards or fused or knobs" --timeout 200 --timeout-method thread > gpurun_out/r03zh/tests_v5.log 2>&1 || { tail -30 gpurun_out/r03zh/tests_v5.log; exit 1; }
tail -1 gpurun_out/r03zh/tests_v5.log
i=0
for n in base v5 base v5; do
  i=$((i+1))
  if [ "$n" = base ]; then L=$PWD/aniso_amd/libaniso_mi355x.so; else L=$PWD/build/ab_$n/libaniso_mi355x.so; fi
  ANISO_LIB=$L timeout -k 10 200 python -u tools/ab_timing.py 60 > gpurun_out/r03zh/abt_${n}_$i.log 2>&1 || { tail -20 gpurun_out/r03zh/abt_${n}_$i.log; exit 1; }
  echo "$n $(grep '^{' gpurun_out/r03zh/abt_${n}_$i.log)"
done
for n in base v5 base v5 base v5; do
  if [ "$n" = base ]; then L=$PWD/aniso_amd/libaniso_mi355x.so; else L=$PWD/build/ab_$n/libaniso_mi355x.so; fi
  ANISO_LIB=$L timeout -k 10 200 python3 tools/shard_time.py 8 0 1 --native --no-timing > gpurun_out/r03zh/w8_$n.log 2>&1 || { tail -20 gpurun_out/r03zh/w8_$n.log; exit 1; }
  echo "$n w8 $(grep '^{' gpurun_out/r03zh/w8_$n.log | cut -c1-90 | tr '\n' ' ')"
done
