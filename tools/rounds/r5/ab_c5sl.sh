#!/bin/bash
# Round 5 A/B: K5 f32 with two C^ slices (3 workgroups per CU) vs three
set -o pipefail
O=gpurun_out/r5_ab_c5sl; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 env AB_CFG=5 python3 tools/ab_lib.py ab/sl0.so,ab/sl2w2.so,ab/base.so 3 8 > $O/c5.txt 2>&1 &&
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_f32.py > $O/parity.txt 2>&1
