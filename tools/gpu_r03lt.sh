#!/bin/bash
# r03lt: parity of the final defaults (fused launch, 128-VGPR near field) over the GPU suite
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03lt
timeout -k 10 900 python -u -m pytest tests/ -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r03lt/tests.log 2>&1 || { tail -40 gpurun_out/r03lt/tests.log; exit 1; }
tail -1 gpurun_out/r03lt/tests.log
