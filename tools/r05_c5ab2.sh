#!/bin/bash
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
AB_CFG=5 timeout -k 10 400 python3 -u tools/ab_env.py TRITD_SB_MAIN -,0 3 8 > gpurun_out/ab_sb.log 2>&1 || exit $?
tail -2 gpurun_out/ab_sb.log
AB_CFG=5 timeout -k 10 400 python3 -u tools/ab_env.py TRITD_GRAM_MAIN -,7 3 8 > gpurun_out/ab_gm.log 2>&1 || exit $?
tail -2 gpurun_out/ab_gm.log
