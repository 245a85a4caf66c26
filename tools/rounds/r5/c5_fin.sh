#!/bin/bash
# Round 5: config-5 finish in M1 + pinv fallback behind the solve (new2) vs
# the side-Gram build (new); trace of new2; then the full GPU suite
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_c5fin; mkdir -p $O
AB_CFG=5 timeout -k 10 500 python3 -u tools/ab_lib.py ab/new.so,ab/new2.so 3 8 > $O/ab.txt 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py --config 5 --no-cpu --no-e2e --no-prims --no-c5 --steps 10 --warmup 3 > $O/line.json 2> $O/err.txt || exit $?
python3 tools/trace_iter.py $O/stats/run_kernel_trace.csv 3 "k5_f32s<" > $O/iter.txt
bash tools/rounds/r5/suite.sh r5_c5fin/suite
