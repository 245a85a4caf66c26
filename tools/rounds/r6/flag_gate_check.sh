#!/bin/bash
# Round 6: the maxIter = 0 pinv-flag test against a library built without the mode-0 gating of the
# solve's pinv fallback (TRITD_NOGATE=1): the test must fail there (it guards ADVICE r5's case).
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6_flag
TRITD_LIB=$PWD/ab6/nogate.so timeout -k 10 300 python3 -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_flags.py -k never_runs > gpurun_out/r6_flag/nogate.txt 2>&1
echo "pytest rc=$?"
