#!/bin/bash
# Round 5: fp32 finish inside M2's first workgroup: f32 tests, config-5 trace
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_m2fin; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_f32.py -x -q --timeout 300 --timeout-method thread > $O/f32_tests.txt 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py --config 5 --no-cpu --no-e2e --no-prims --no-c5 --steps 10 --warmup 3 > $O/c5_line.json 2> $O/c5_err.txt || exit $?
python3 tools/trace_iter.py $O/stats/run_kernel_trace.csv 3 "k5_f32s<" > $O/c5_iter.txt
python3 tools/trace_iter.py $O/stats/run_kernel_trace.csv 5 "k5_f32s<" >> $O/c5_iter.txt
