#!/bin/bash
# r03q: 8-shard rank time: serial vs overlapped near field, cluster depth 1, ring form
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03q
timeout -k 10 400 python -u tools/ab_handles.py --world 8 --reps 4 "" "ANISO_OVERLAP=0" "ANISO_HM_CLDEPTH=1" "ANISO_HM_CLDEPTH=1,ANISO_OVERLAP=0" "ANISO_HM_RING=3" "ANISO_HM_RING=3,ANISO_OVERLAP=0" > gpurun_out/r03q/ab_w8.log 2>&1 || { tail -20 gpurun_out/r03q/ab_w8.log; exit 1; }
grep "^{" gpurun_out/r03q/ab_w8.log | cut -c1-330
