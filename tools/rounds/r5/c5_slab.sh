#!/bin/bash
# Round 5: f32 K2 slabs + vectorised apply (new4) vs new3; parity tests; trace
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_slab; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_f32.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
AB_CFG=5 timeout -k 10 500 python3 -u tools/ab_lib.py ab/new3.so,ab/new4.so 3 8 > $O/ab.txt 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py --config 5 --no-cpu --no-e2e --no-prims --no-c5 --steps 10 --warmup 3 > $O/line.json 2> $O/err.txt || exit $?
python3 tools/trace_iter.py $O/stats/run_kernel_trace.csv 3 "k5_f32s<" > $O/iter.txt
