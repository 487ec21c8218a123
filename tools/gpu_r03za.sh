#!/bin/bash
# r03za: HEAD of round 3 (down-pass task records in LDS, 128-VGPR near field): smoke, kernel trace + stats, FETCH/WRITE passes, bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03za
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03za/smoke.log 2>&1 || { tail -20 gpurun_out/r03za/smoke.log; exit 1; }
tail -2 gpurun_out/r03za/smoke.log
bash tools/profile_round.sh r03za || exit $?
python3 tools/pmc_summary.py gpurun_out/prof_r03za/fetch/run_counter_collection.csv gpurun_out/prof_r03za/write/run_counter_collection.csv gpurun_out/r03za/pmc_summary.json || exit 1
python3 tools/trace_last.py gpurun_out/prof_r03za/trace/run_kernel_trace.csv > gpurun_out/r03za/timeline_w1.txt || exit 1
cat gpurun_out/r03za/timeline_w1.txt
timeout -k 10 600 python bench.py > gpurun_out/r03za/bench.log 2>&1 || { tail -20 gpurun_out/r03za/bench.log; exit 1; }
grep "^{" gpurun_out/r03za/bench.log | tail -1 | cut -c1-600
