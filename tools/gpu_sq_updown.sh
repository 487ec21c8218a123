#!/bin/bash
# SQ + TA/TD counter passes of a short bench run (up/down/M2L/near kernels).
# usage: bash tools/gpu_sq_updown.sh <tag>
set -o pipefail
TAG=${1:-ud}
bash tools/sq_profile.sh $TAG || exit $?
OUT=gpurun_out/sq_$TAG
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/p3 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $OUT/p3.log 2>&1 || exit $?
python3 tools/sq_summary.py $TAG
