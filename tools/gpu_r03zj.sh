#!/bin/bash
# r03zj: HEAD with the dynamic target hand-out: in-process knob A/B (cluster occupancy
# and near-field VGPR cap re-checked), then kernel trace + stats, FETCH/WRITE passes
# and the bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03zj
timeout -k 10 400 python -u tools/ab_handles.py --reps 4 "" "ANISO_HM_WPE=8" "ANISO_NEAR_WPE=3" "ANISO_HM_WPE=8,ANISO_NEAR_WPE=3" > gpurun_out/r03zj/ab_w1.log 2>&1 || { tail -20 gpurun_out/r03zj/ab_w1.log; exit 1; }
grep "^{" gpurun_out/r03zj/ab_w1.log | cut -c1-300
bash tools/profile_round.sh r03zj || exit $?
python3 tools/pmc_summary.py gpurun_out/prof_r03zj/fetch/run_counter_collection.csv gpurun_out/prof_r03zj/write/run_counter_collection.csv gpurun_out/r03zj/pmc_summary.json > /dev/null || exit 1
python3 tools/trace_last.py gpurun_out/prof_r03zj/trace/run_kernel_trace.csv > gpurun_out/r03zj/timeline_w1.txt || exit 1
cat gpurun_out/r03zj/timeline_w1.txt
timeout -k 10 600 python bench.py > gpurun_out/r03zj/bench.log 2>&1 || { tail -20 gpurun_out/r03zj/bench.log; exit 1; }
grep "^{" gpurun_out/r03zj/bench.log | tail -1 | cut -c1-300
