# sharded-exchange tests, then one rank-of-8 schedule (loopback) with the upper
# multipoles as partial sums on and off: ms per apply without stage events, then stages
set -o pipefail
T=${TAG:-r05}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "${TESTS:-native_exchange}" > gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/shard_time.py 8 0 3 5 7 --native --no-timing > gpurun_out/${T}_shard_on.log 2>&1 && \
ANISO_UPPER_PARTIAL=0 timeout -k 10 300 python -u tools/shard_time.py 8 0 3 5 7 --native --no-timing > gpurun_out/${T}_shard_off.log 2>&1 && \
timeout -k 10 300 python -u tools/shard_time.py 8 0 3 --native > gpurun_out/${T}_shard_on_stages.log 2>&1
