#!/bin/bash
# r03ze: the staged near field with one Newton step after v_rsq_f64 (build/ab_v4,
# -DANISO_NEAR_NR=1; the M2L already runs one) against the in-tree build (two):
# parity subset on v4 (block matvec vs oracle and vs mode applies), wall time alternating
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03ze
L1=$PWD/build/ab_v4/libaniso_mi355x.so
ANISO_LIB=$L1 timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "clusters_match or config3_size_matches or block_operator_matches or eight_shards or fused or knobs or sz512 or block_solve or harmonic" --timeout 200 --timeout-method thread > gpurun_out/r03ze/tests_v4.log 2>&1 || { tail -30 gpurun_out/r03ze/tests_v4.log; exit 1; }
tail -1 gpurun_out/r03ze/tests_v4.log
i=0
for n in base v4 base v4; do
  i=$((i+1))
  if [ "$n" = base ]; then L=$PWD/aniso_amd/libaniso_mi355x.so; else L=$PWD/build/ab_$n/libaniso_mi355x.so; fi
  ANISO_LIB=$L timeout -k 10 200 python -u tools/ab_timing.py 60 > gpurun_out/r03ze/abt_${n}_$i.log 2>&1 || { tail -20 gpurun_out/r03ze/abt_${n}_$i.log; exit 1; }
  echo "$n $(grep '^{' gpurun_out/r03ze/abt_${n}_$i.log)"
done
for n in base v4 base v4; do
  if [ "$n" = base ]; then L=$PWD/aniso_amd/libaniso_mi355x.so; else L=$PWD/build/ab_$n/libaniso_mi355x.so; fi
  ANISO_LIB=$L timeout -k 10 200 python3 tools/shard_time.py 8 0 1 --native --no-timing > gpurun_out/r03ze/w8_$n.log 2>&1 || { tail -20 gpurun_out/r03ze/w8_$n.log; exit 1; }
  echo "$n w8 $(grep '^{' gpurun_out/r03ze/w8_$n.log | cut -c1-90 | tr '\n' ' ')"
done
