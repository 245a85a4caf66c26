#!/bin/bash
# Round 5 A/B: fp32 K2 (B^ two fibres ahead) and Gram side jobs at any size
set -o pipefail
O=gpurun_out/r5_ab_k2g; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 env AB_CFG=5 python3 tools/ab_lib.py ab/c5new.so,ab/c5k2.so 3 8 > $O/c5.txt 2>&1 &&
timeout -k 10 200 python3 tools/ab_lib.py ab/gsmall.so,ab/gany.so 3 10 > $O/c4.txt 2>&1 &&
timeout -k 10 120 env TRITD_LIB=ab/gsmall.so python3 tools/shard_timing.py 8 > $O/shard_small.txt 2>&1 &&
timeout -k 10 120 env TRITD_LIB=ab/gany.so python3 tools/shard_timing.py 8 > $O/shard_any.txt 2>&1 &&
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_f32.py tests/test_gpu_configs.py > $O/parity.txt 2>&1
