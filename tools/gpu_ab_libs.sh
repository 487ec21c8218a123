#!/bin/bash
# A/B of library builds (tools/build_variant.sh): block-matvec parity subset, then the
# wall time with and without stage events (tools/ab_timing.py) per build.
# usage: tools/gpu_ab_libs.sh <tag> <name>...   (name "base" = the in-tree library)
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in "$@"; do
  if [ "$n" = base ]; then L=$PWD/aniso_amd/libaniso_mi355x.so; else L=$PWD/build/ab_$n/libaniso_mi355x.so; fi
  ANISO_LIB=$L timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "clusters_match or config3_size_matches or block_operator_matches or eight_shards" --timeout 200 --timeout-method thread > gpurun_out/ab_${TAG}_$n.log 2>&1 || { tail -30 gpurun_out/ab_${TAG}_$n.log; exit 1; }
  tail -1 gpurun_out/ab_${TAG}_$n.log
  for r in 1 2; do
    ANISO_LIB=$L timeout -k 10 200 python -u tools/ab_timing.py 60 > gpurun_out/abt_${TAG}_${n}_$r.log 2>&1 || { tail -20 gpurun_out/abt_${TAG}_${n}_$r.log; exit 1; }
    echo "$n $(grep '^{' gpurun_out/abt_${TAG}_${n}_$r.log)"
  done
done
