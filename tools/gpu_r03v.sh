#!/bin/bash
# r03v: smoke, kernel trace + stats and the FETCH/WRITE passes of bench.py, then the bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03v
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03v/smoke.log 2>&1 || { tail -20 gpurun_out/r03v/smoke.log; exit 1; }
tail -2 gpurun_out/r03v/smoke.log
bash tools/profile_round.sh r03v || exit $?
python3 tools/pmc_summary.py gpurun_out/prof_r03v/fetch/run_counter_collection.csv gpurun_out/prof_r03v/write/run_counter_collection.csv gpurun_out/r03v/pmc_summary.json || exit 1
python3 tools/trace_last.py gpurun_out/prof_r03v/trace/run_kernel_trace.csv > gpurun_out/r03v/timeline_w1.txt || exit 1
cat gpurun_out/r03v/timeline_w1.txt
timeout -k 10 600 python bench.py > gpurun_out/r03v/bench.log 2>&1 || { tail -20 gpurun_out/r03v/bench.log; exit 1; }
grep "^{" gpurun_out/r03v/bench.log | tail -1 | cut -c1-600
