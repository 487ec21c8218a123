#!/bin/bash
# r03c: staged-source M2L with 4-wave workgroups and 16-target clusters vs the others
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_handles.py "ANISO_OVERLAP=0,ANISO_HM_STAGED=0" "ANISO_OVERLAP=0,ANISO_CS_WAVES=4,ANISO_HM_CLDEPTH=2" "ANISO_OVERLAP=0,ANISO_HM_STAGED=0,ANISO_HM_CLDEPTH=2" "ANISO_CS_WAVES=4,ANISO_HM_CLDEPTH=2" "ANISO_HM_STAGED=0" > gpurun_out/ab_r03c.log 2>&1 || { tail -20 gpurun_out/ab_r03c.log; exit 1; }
cat gpurun_out/ab_r03c.log
timeout -k 10 300 python -u tools/ab_handles.py --world 8 "ANISO_OVERLAP=0,ANISO_HM_STAGED=0" "ANISO_OVERLAP=0,ANISO_CS_WAVES=4" "ANISO_HM_STAGED=0" "ANISO_CS_WAVES=4" > gpurun_out/ab8_r03c.log 2>&1 || { tail -20 gpurun_out/ab8_r03c.log; exit 1; }
cat gpurun_out/ab8_r03c.log
