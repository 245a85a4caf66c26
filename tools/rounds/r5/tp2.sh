#!/bin/bash
# Round 5: triple product with two ij-tiles per wave (tp2) vs one (tp1): parity tests, primitives A/B
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_tp2; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_devprod.py tests/test_gpu_parity.py tests/test_gpu_metrics.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/ab_prims.py ab/tp1.so ab/tp2.so 5 > $O/ab.txt 2>&1
