#!/bin/bash
# Round 5: cause of the round-4 K5 store corruption.
#  1. the probe: wide-store data rewritten at 0 / 1 wait states, per store form
#  2. the library built with TRITD_STORE_KEEP=0 (ab/nokeep) on the bitwise
#     repeat tests (expected to fail), then the product build (expected to pass)
O=gpurun_out/r5_hazard
mkdir -p $O
timeout -k 10 120 tools/store_hazard.bin > $O/probe.txt 2>&1 || exit $?
TRITD_LIB=ab/nokeep/libtritd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_determinism.py \
    -k "config3 or traffic" -v --timeout 300 --timeout-method thread > $O/nokeep_tests.txt 2>&1
rc=$?
echo "nokeep rc=$rc" >> $O/nokeep_tests.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_determinism.py -k "config3 or traffic" -v \
    --timeout 300 --timeout-method thread > $O/keep_tests.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $O/bench.txt 2>&1
