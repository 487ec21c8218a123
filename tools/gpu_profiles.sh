# the round's profiles on one box: bench kernel trace + stats and PMC passes, then the
# 16-RHS MFMA operators' counters (tools/profile_round.sh, f32op_prof.sh, f64op_prof.sh)
set -o pipefail
T=${1:-r05}
bash tools/profile_round.sh $T > gpurun_out/${T}_profile_round.log 2>&1 || exit $?
python3 tools/pmc_summary.py $(find gpurun_out/prof_$T/fetch -name "*counter_collection.csv") $(find gpurun_out/prof_$T/write -name "*counter_collection.csv") gpurun_out/prof_$T/pmc_summary.json || exit $?
bash tools/f32op_prof.sh $T > gpurun_out/${T}_f32op_prof.log 2>&1 || exit $?
bash tools/f64op_prof.sh $T > gpurun_out/${T}_f64op_prof.log 2>&1
