#!/bin/bash
# Round 6, final build: the whole GPU suite, smoke(), and the default bench line (one MI355X).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_suite; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread > $O/gpu_tests_full.log.txt 2>&1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log.txt 2>&1
timeout -k 10 600 python3 bench.py > $O/bench_line.json 2> $O/bench.err
echo done
