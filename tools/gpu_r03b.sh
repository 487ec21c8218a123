#!/bin/bash
# r03b: staged-source M2L A/B at 1 GPU and one rank of 8
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_handles.py "" "ANISO_HM_STAGED=0" "ANISO_OVERLAP=0" "ANISO_OVERLAP=0,ANISO_HM_STAGED=0" > gpurun_out/ab_r03b.log 2>&1 || { tail -20 gpurun_out/ab_r03b.log; exit 1; }
cat gpurun_out/ab_r03b.log
timeout -k 10 300 python -u tools/ab_handles.py --world 8 "" "ANISO_HM_STAGED=0" "ANISO_OVERLAP=0" "ANISO_OVERLAP=0,ANISO_HM_STAGED=0" > gpurun_out/ab8_r03b.log 2>&1 || { tail -20 gpurun_out/ab8_r03b.log; exit 1; }
cat gpurun_out/ab8_r03b.log
