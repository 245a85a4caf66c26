#!/bin/bash
# Round 6: config-5 K5 (k5_f32s) with its C^ operand reads issued ahead (all eight L reads before the
# first L MFMA, the W reads of row r+1 before the MFMAs of row r) — bitwise equality at config 5,
# fp32 parity with the variant library, interleaved A/B at config 5.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_lpre; mkdir -p $O
AB_CFG=5 timeout -k 10 300 python3 -u tools/ab_same.py ab6/base.so,ab6/lpre.so 0 16 6 > $O/same_c5.txt 2>&1
AB_CFG=5 timeout -k 10 700 python3 -u tools/ab_lib.py ab6/base.so,ab6/lpre.so 4 6 > $O/ab_c5.txt 2>&1
TRITD_LIB=$PWD/ab6/lpre.so timeout -k 10 900 python3 -u -m pytest -x -v --timeout 800 --timeout-method thread -m gpu \
    tests/test_gpu_f32.py tests/test_gpu_fullsize.py tests/test_gpu_determinism.py -k "f32 or config5" > $O/parity.txt 2>&1
echo done
