#!/bin/bash
# One config-4 iteration's kernel timeline (rocprofv3 kernel trace of a short bench)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/p1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/p1/trace -o run -- \
    python3 bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/p1/trace.log 2>&1 || exit $?
python3 tools/trace_iter.py gpurun_out/p1/trace/run_kernel_trace.csv 60
