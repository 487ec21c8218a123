#!/bin/bash
# r03r: full GPU suite after the ring / timeline work
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03r
timeout -k 10 1000 python -u -m pytest tests/ -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r03r/tests.log 2>&1 || { tail -40 gpurun_out/r03r/tests.log; exit 1; }
tail -3 gpurun_out/r03r/tests.log
