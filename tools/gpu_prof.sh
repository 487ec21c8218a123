set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r01h}
bash tools/profile_round.sh $TAG || exit $?
python3 tools/pmc_summary.py $(find gpurun_out/prof_$TAG/fetch -name "*counter_collection.csv") $(find gpurun_out/prof_$TAG/write -name "*counter_collection.csv") gpurun_out/prof_$TAG/pmc_summary.json || exit $?
