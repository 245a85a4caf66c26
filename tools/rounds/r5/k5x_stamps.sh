#!/bin/bash
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_stamps; mkdir -p $O
AB_CFG=5 TRITD_K5X_STAMPS=$O/st.bin timeout -k 10 300 python3 -u tools/ab_lib.py ab/stamps.so 1 8 > $O/ab.txt 2>&1 &&
python3 tools/rounds/r5/k5x_stamps.py $O/st.bin > $O/summary.txt 2>&1
