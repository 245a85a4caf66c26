#!/bin/bash
# Round 6: fp32 compact-E encode with one select per element — fp32 parity (bitwise repeat included)
# with the new library, interleaved A/B at config 5.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_enc32; mkdir -p $O
TRITD_LIB=$PWD/ab6/new.so timeout -k 10 900 python3 -u -m pytest -x -v --timeout 800 --timeout-method thread -m gpu \
    tests/test_gpu_f32.py tests/test_gpu_fullsize.py tests/test_gpu_determinism.py -k "f32 or config5" > $O/parity.txt 2>&1
AB_CFG=5 timeout -k 10 600 python3 -u tools/ab_lib.py ab6/base.so,ab6/new.so 3 6 > $O/ab_c5.txt 2>&1
echo done
