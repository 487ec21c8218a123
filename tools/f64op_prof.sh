#!/bin/bash
# The fp64 16-RHS MFMA operator under rocprofv3: kernel trace + stats, then separate
# PMC passes: fp64 MFMA instructions / busy cycles (SQ + GRBM), FETCH_SIZE, WRITE_SIZE.
# usage: bash tools/f64op_prof.sh <tag>
set -o pipefail
TAG=${1:-f64}
OUT=gpurun_out/f64prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/f64op_bench.py 1024 20 > $OUT/trace.log 2>&1 || exit $?
grep "^{" $OUT/trace.log
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/mfma -o run -- python3 tools/f64op_bench.py 1024 5 > $OUT/mfma.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 tools/f64op_bench.py 1024 5 > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 tools/f64op_bench.py 1024 5 > $OUT/write.log 2>&1 || exit $?
python3 tools/pmc_summary.py $(find $OUT/fetch -name "*counter_collection.csv") $(find $OUT/write -name "*counter_collection.csv") $OUT/pmc_summary.json || exit $?
python3 tools/counter_summary.py $(find $OUT/mfma -name "*counter_collection.csv") $OUT/mfma_summary.json
