set -uo pipefail
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
SHARD_MODES=rccl-sharded timeout -k 10 300 python3 tools/shard_timing.py 2 2 2 1 4 > gpurun_out/p2.log 2>&1; cat gpurun_out/p2.log | grep "P="
