#!/bin/bash
# L2 / HBM counter passes of a short bench run (one counter group per pass).
# usage: bash tools/pmc_l2.sh <tag> [ENV=VAL ...]
set -o pipefail
TAG=${1:-l2}
shift
OUT=gpurun_out/l2_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
i=0
for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $OUT/p$i.log 2>&1 || exit $?
done
python3 tools/sq_summary.py l2_$TAG | grep -A1 "k_m2l\|k_near"
