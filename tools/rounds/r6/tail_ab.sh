#!/bin/bash
# Round 6: config-4 iteration tail — M1 (two rows per lane, JS slices) and M2 (j per wave) A/B,
# plus one bench kernel trace of the iteration.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_tail; mkdir -p $O
TRITD_M1_V=8 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "golden or shards or first" > $O/m1v8_parity.txt 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/m1prof -o run -- \
    python3 tools/ab_env.py TRITD_M1_V -,4,8,16 3 20 > $O/m1_ab.txt 2>&1
timeout -k 10 400 python3 tools/ab_lib.py ab6/base.so,ab6/m2j2.so,ab6/m2j4.so 3 20 > $O/m2_ab.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- \
    python3 bench.py --no-cpu --no-e2e --no-prims --no-c5 --steps 10 --warmup 2 > $O/trace.log 2>&1
python3 tools/trace_iter.py $O/trace/run_kernel_trace.csv 3 > $O/iter.txt
echo done
