#!/bin/bash
# Round 6, last commit: the whole GPU suite and smoke() (no bench / PMC: the kernels are those of
# tools/rounds/r6/final_all.sh's run; this adds the flags test and the grouped all-reduce change).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_suite_head; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread > $O/gpu_tests_full.log.txt 2>&1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log.txt 2>&1
echo done
