#!/bin/bash
# r03zf: round-3 close at HEAD: the whole -m gpu suite, smoke, kernel trace + stats and
# the FETCH/WRITE passes of bench.py, then the bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03zf
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r03zf/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r03zf/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03zf/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03zf/smoke.log 2>&1 || { tail -20 gpurun_out/r03zf/smoke.log; exit 1; }
tail -1 gpurun_out/r03zf/smoke.log
bash tools/profile_round.sh r03zf || exit $?
python3 tools/pmc_summary.py gpurun_out/prof_r03zf/fetch/run_counter_collection.csv gpurun_out/prof_r03zf/write/run_counter_collection.csv gpurun_out/r03zf/pmc_summary.json > /dev/null || exit 1
python3 tools/trace_last.py gpurun_out/prof_r03zf/trace/run_kernel_trace.csv > gpurun_out/r03zf/timeline_w1.txt || exit 1
cat gpurun_out/r03zf/timeline_w1.txt
timeout -k 10 600 python bench.py > gpurun_out/r03zf/bench.log 2>&1 || { tail -20 gpurun_out/r03zf/bench.log; exit 1; }
grep "^{" gpurun_out/r03zf/bench.log | tail -1 | cut -c1-400
