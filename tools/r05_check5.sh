#!/bin/bash
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mex_gateway.py tests/test_gpu_parity.py tests/test_gpu_metrics.py tests/test_drivers.py tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/t5.log 2>&1
rc=$?; tail -1 gpurun_out/t5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/bench_prims.py > gpurun_out/prims.json 2> gpurun_out/prims.err || exit $?
cut -c1-600 gpurun_out/prims.json
