#!/bin/bash
# Round 5: config-5 K5 variants (prologue order / persistent grid) A/B, their
# fp32 parity, and the P=8 shard timing of the current build.
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_ab_c5; mkdir -p $O
AB_CFG=5 timeout -k 10 500 python3 -u tools/ab_lib.py ab/c5old.so,ab/c5new.so,ab/c5persist.so 3 8 > $O/ab.txt 2>&1 || exit $?
for v in c5new c5persist; do
  TRITD_LIB=ab/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_determinism.py \
      -x -q --timeout 300 --timeout-method thread -k "f32" > $O/tests_$v.txt 2>&1
  rc=$?; echo "rc=$rc" >> $O/tests_$v.txt; [ $rc -le 1 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/shard -o run -- \
    python3 tools/shard_timing.py 8 4 > $O/shard.txt 2>&1
