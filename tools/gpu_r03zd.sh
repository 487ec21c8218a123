#!/bin/bash
# r03zd: quad-shared multipole loads in the cluster M2L (build/ab_v2: each lane of a
# quad loads ceil(K/4) entries, DPP broadcasts the rest) against the in-tree build:
# parity subset on v2, wall time alternating; rank 0 of 8 (loopback)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03zd
L1=$PWD/build/ab_v2/libaniso_mi355x.so
ANISO_LIB=$L1 timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "clusters_match or config3_size_matches or block_operator_matches or eight_shards or fused or knobs" --timeout 200 --timeout-method thread > gpurun_out/r03zd/tests_v2.log 2>&1 || { tail -30 gpurun_out/r03zd/tests_v2.log; exit 1; }
tail -1 gpurun_out/r03zd/tests_v2.log
i=0
for n in base v2 base v2; do
  i=$((i+1))
  if [ "$n" = base ]; then L=$PWD/aniso_amd/libaniso_mi355x.so; else L=$PWD/build/ab_$n/libaniso_mi355x.so; fi
  ANISO_LIB=$L timeout -k 10 200 python -u tools/ab_timing.py 60 > gpurun_out/r03zd/abt_${n}_$i.log 2>&1 || { tail -20 gpurun_out/r03zd/abt_${n}_$i.log; exit 1; }
  echo "$n $(grep '^{' gpurun_out/r03zd/abt_${n}_$i.log)"
done
for n in base v2 base v2; do
  if [ "$n" = base ]; then L=$PWD/aniso_amd/libaniso_mi355x.so; else L=$PWD/build/ab_$n/libaniso_mi355x.so; fi
  ANISO_LIB=$L timeout -k 10 200 python3 tools/shard_time.py 8 0 1 --native --no-timing > gpurun_out/r03zd/w8_$n.log 2>&1 || { tail -20 gpurun_out/r03zd/w8_$n.log; exit 1; }
  echo "$n w8 $(grep '^{' gpurun_out/r03zd/w8_$n.log | cut -c1-90 | tr '\n' ' ')"
done
