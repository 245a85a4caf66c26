#!/bin/bash
# Round 6: K5's chain through dE = E^(k) - E^(k-1) (D - L from the MFMA chain) — parity with the
# variant library, then an interleaved iteration A/B.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_dl; mkdir -p $O
TRITD_LIB=$PWD/ab6/dl.so timeout -k 10 700 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_determinism.py -k "not config5" > $O/parity.txt 2>&1
timeout -k 10 500 python3 tools/ab_lib.py ab6/base.so,ab6/dl.so 6 20 > $O/ab_c4.txt 2>&1
echo done
