#!/bin/bash
# Round 6: K2 (k_m3_cp) with two prefetch register sets used in turn instead of a per-step copy
# (no v_mov_b64 in the loop) — bitwise equality, parity with the variant library, interleaved A/B.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_k2pp; mkdir -p $O
timeout -k 10 300 python3 tools/ab_same.py ab6/base.so,ab6/pp.so 256 8 12 > $O/same.txt 2>&1
timeout -k 10 300 python3 tools/ab_same.py ab6/base.so,ab6/pp.so 96 5 30 > $O/same_small.txt 2>&1
TRITD_LIB=$PWD/ab6/pp.so timeout -k 10 700 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py tests/test_gpu_determinism.py tests/test_gpu_dist_host.py -k "not config5" > $O/parity.txt 2>&1
timeout -k 10 500 python3 tools/ab_lib.py ab6/base.so,ab6/pp.so 6 20 > $O/ab_c4.txt 2>&1
echo done
