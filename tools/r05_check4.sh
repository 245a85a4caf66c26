#!/bin/bash
# host-transport multi-rank tests, fp32 / large-rank parity, config-5 bench
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_host.py tests/test_gpu_f32.py tests/test_gpu_parity.py tests/test_drivers.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_t4.log 2>&1
rc=$?; grep -E "passed|failed|FAIL|Error" gpurun_out/gpu_t4.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --config 5 --no-cpu --no-e2e --steps 10 --warmup 3 > gpurun_out/bench5.json 2> gpurun_out/bench5.err || exit $?
cut -c1-900 gpurun_out/bench5.json
