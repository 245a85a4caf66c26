#!/bin/bash
# Round 6: config-5 K2 (k_m3_32<256>) with the Khatri-Rao formation at immediate LDS offsets (176 -> 148
# VGPRs: three workgroups per CU) — fp32 parity, interleaved A/B, fibre-chunk count A/B.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_c5k2; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 800 --timeout-method thread -m gpu \
    tests/test_gpu_f32.py tests/test_gpu_fullsize.py -k "f32 or config5" > $O/parity.txt 2>&1
AB_CFG=5 timeout -k 10 600 python3 -u tools/ab_lib.py ab6/old.so,ab6/new.so 3 6 > $O/ab_c5.txt 2>&1
AB_CFG=5 timeout -k 10 600 python3 -u tools/ab_env.py TRITD_M3_JC -,3,6 2 6 > $O/ab_jc.txt 2>&1
echo done
