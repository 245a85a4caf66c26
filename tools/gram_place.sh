#!/bin/bash
# Gram placement sweep: 1-GPU overlapped schedule (TRITD_GRAM_MAIN) and the
# P = 8 shard of the sharded schedule (TRITD_GRAM_MAIN_SH), bits 0 A, 1 B, 2 C.
set -uo pipefail
for gm in 0 2 4 6; do
  echo "GRAM_MAIN=$gm"; TRITD_GRAM_MAIN=$gm OVS=3 timeout -k 10 200 python3 tools/timing_overhead.py 2>&1 | grep "timing=0" | tail -1 || exit 1
done
for gm in 0 2 4 6; do
  echo "GRAM_MAIN_SH=$gm"; TRITD_GRAM_MAIN_SH=$gm SHARD_MODES=rccl-sharded timeout -k 10 200 python3 tools/shard_timing.py 8 2>&1 | grep "P=" || exit 1
done
