#!/bin/bash
# Round 6: both K5 walks (k5_fused, k5_f32s) with __builtin_amdgcn_iglp_opt(0) in the t-tile body (LLVM's
# MFMA / DS-read interleave) — bitwise equality, interleaved A/Bs at configs 4 and 5.  (iglp_opt(1) runs
# the compiler out of memory on k_admm.hip.)
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_iglp; mkdir -p $O
timeout -k 10 300 python3 tools/ab_same.py ab6/base.so,ab6/ig0.so 256 8 12 > $O/same.txt 2>&1
AB_CFG=5 timeout -k 10 300 python3 -u tools/ab_same.py ab6/base.so,ab6/ig0.so 0 16 4 > $O/same_c5.txt 2>&1
timeout -k 10 500 python3 tools/ab_lib.py ab6/base.so,ab6/ig0.so 6 20 > $O/ab_c4.txt 2>&1
AB_CFG=5 timeout -k 10 600 python3 -u tools/ab_lib.py ab6/base.so,ab6/ig0.so 3 6 > $O/ab_c5.txt 2>&1
echo done
