# the round's closing checks on one box: GPU suite, smoke(), the default bench command
set -o pipefail
T=${1:-r05}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.log 2>&1
