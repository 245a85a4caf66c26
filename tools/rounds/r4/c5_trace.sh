#!/bin/bash
# One config-5 iteration's kernel timeline (rocprofv3 kernel trace of a short bench)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c5t
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c5t/trace -o run -- \
    python3 bench.py --config 5 --no-cpu --no-e2e --steps 4 --warmup 2 > gpurun_out/c5t/trace.log 2>&1 || exit $?
python3 tools/trace_iter.py gpurun_out/c5t/trace/run_kernel_trace.csv 8 "k5_f32s<" > gpurun_out/c5t/iter.txt
cat gpurun_out/c5t/iter.txt
