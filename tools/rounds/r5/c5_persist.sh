#!/bin/bash
# Round 5: persistent K5 f32 (k5_f32p) — errHist vs k5_f32s, fp32 tests, config-5 A/B
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_persist; mkdir -p $O
ITERS=100 timeout -k 10 300 python3 -u tools/rounds/r5/cmp_eh.py ab/new3.so ab/p1.so > $O/eh.txt 2>&1 || exit $?
TRITD_LIB=ab/p1.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_f32.py -x -q --timeout 300 --timeout-method thread > $O/tests_p1.txt 2>&1 || exit $?
AB_CFG=5 timeout -k 10 500 python3 -u tools/ab_lib.py ab/new3.so,ab/p1.so,ab/p2.so 3 8 > $O/ab.txt 2>&1
