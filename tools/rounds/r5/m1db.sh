#!/bin/bash
# Round 5: fp64 M1 with its next load batch in flight (m1db) vs before (old): config 4, P = 8 shard, parity
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_m1db; mkdir -p $O
timeout -k 10 400 python3 -u tools/ab_lib.py ab/old.so,ab/m1db.so 4 10 > $O/ab.txt 2>&1 || exit $?
for v in old m1db old m1db; do TRITD_LIB=ab/$v.so timeout -k 10 100 python3 tools/shard_timing.py 8 2>&1 | grep "P=" | sed "s/^/$v /" >> $O/shard.txt || exit $?; done
TRITD_LIB=ab/m1db.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_determinism.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
