# one box, one call: the round's bench profiles (kernel trace + stats, PMC passes), then
# the closing checks (GPU suite, smoke(), the default bench command)
# usage: bash tools/gpu_close.sh <profile tag> <check tag>
set -o pipefail
P=${1:-r05p}
C=${2:-r05c}
bash tools/profile_round.sh $P > gpurun_out/${P}_profile_round.log 2>&1 || exit $?
python3 tools/pmc_summary.py $(find gpurun_out/prof_$P/fetch -name "*counter_collection.csv") $(find gpurun_out/prof_$P/write -name "*counter_collection.csv") gpurun_out/prof_$P/pmc_summary.json > gpurun_out/${P}_pmc.log 2>&1 || exit $?
bash tools/gpu_final.sh $C
