set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/profile_round.sh r01f || exit $?
python3 tools/pmc_summary.py $(find gpurun_out/prof_r01f/fetch -name "*counter_collection.csv") $(find gpurun_out/prof_r01f/write -name "*counter_collection.csv") gpurun_out/prof_r01f/pmc_summary.json || exit $?
bash tools/sq_profile.sh hc || exit $?
