#!/bin/bash
# Kernel trace of the unsharded block matvec (bench.py --no-cpu, 1 GPU); ANISO_LIB
# selects an alternative library build for A/B.  usage: gpu_w1prof.sh <tag> [lib]
set -o pipefail
TAG=${1:-w1}
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$2" ] && cd $2 && mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/w1prof_$TAG -o run -- python3 bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/w1prof_$TAG.log 2>&1 || { tail -20 gpurun_out/w1prof_$TAG.log; exit 1; }
grep "^{" gpurun_out/w1prof_$TAG.log | cut -c1-200
python3 $GRAFT_REPO_ROOT/tools/trace_last.py gpurun_out/w1prof_$TAG/run_kernel_trace.csv
