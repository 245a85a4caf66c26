#!/bin/bash
# Round 5: K5 compact-E mask form (K5_CE_V2) and 6 slice buffers, A/B against
# the product build, then parity of the variants; config-5 walk-length probe.
set -uo pipefail
O=gpurun_out/r5_ab_ce; mkdir -p $O
timeout -k 10 300 python3 -u tools/ab_lib.py ab/base.so,ab/v2.so,ab/v2nb6.so 4 10 > $O/ab.txt 2>&1 || exit $?
for v in v2 v2nb6; do
  TRITD_LIB=ab/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_determinism.py tests/test_gpu_parity.py \
      -x -q --timeout 240 --timeout-method thread > $O/tests_$v.txt 2>&1
  rc=$?; echo "rc=$rc" >> $O/tests_$v.txt; [ $rc -le 1 ] || exit $rc
done
timeout -k 10 300 python3 -u tools/c5_walk.py > $O/c5_walk.txt 2>&1
