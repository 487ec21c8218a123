#!/bin/bash
# r03sq: SQ counter passes on a short bench run (instruction mix and stall buckets per kernel)
set -o pipefail
export TMPDIR=/tmp
bash tools/sq_profile.sh r03 --no-solve --gmres 0 --config4-sz 0 || exit 1
python3 tools/sq_summary.py r03 > gpurun_out/sq_r03/summary.txt || exit 1
grep -A1 "k_top_m2l_hc\|k_near_hs\|k_up_tier<5>\|k_down_tier<5>" gpurun_out/sq_r03/summary.txt
