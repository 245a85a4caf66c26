#!/bin/bash
# Round 6, last build: the whole GPU suite, then the PMC / stats evidence, smoke() and the default
# bench line on the same box (tools/rounds/r6/final_profiles2.sh with its output under $O, default r6_final5).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${FINAL_OUT:-gpurun_out/r6_final5}
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread > $O/gpu_tests_full.log.txt 2>&1
sed -e "s|O=gpurun_out/r6_final2;|O=$O;|" tools/rounds/r6/final_profiles2.sh > $O/fp.sh
bash $O/fp.sh
