#!/bin/bash
# SQ counter passes (no traces) on a short bench run: instruction mix and stall
# buckets per kernel.  usage: bash tools/sq_profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-sq}
shift
OUT=gpurun_out/sq_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $OUT/p1 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu "$@" > $OUT/p1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD --output-format csv -d $OUT/p2 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu "$@" > $OUT/p2.log 2>&1 || exit $?
