#!/bin/bash
# Round 6: the whole library compiled with LLVM's max-ilp / max-memory-clause machine schedulers
# (-mllvm -amdgpu-sched-strategy=...) against the default — bitwise equality, parity with each,
# interleaved A/Bs at configs 4 and 5.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_sched; mkdir -p $O
timeout -k 10 300 python3 tools/ab_same.py ab6/base.so,ab6/ilp.so,ab6/mem.so 256 8 12 > $O/same.txt 2>&1
AB_CFG=5 timeout -k 10 300 python3 -u tools/ab_same.py ab6/base.so,ab6/ilp.so,ab6/mem.so 0 16 4 > $O/same_c5.txt 2>&1
timeout -k 10 600 python3 tools/ab_lib.py ab6/base.so,ab6/ilp.so,ab6/mem.so 5 20 > $O/ab_c4.txt 2>&1
AB_CFG=5 timeout -k 10 700 python3 -u tools/ab_lib.py ab6/base.so,ab6/ilp.so,ab6/mem.so 3 6 > $O/ab_c5.txt 2>&1
echo done
