#!/bin/bash
# parity subset (with $PAR_LIB if set, else the in-tree lib), then an
# interleaved A/B of built variants
#   [PAR_LIB=ab/x.so] bash tools/ab_run.sh "ab/base.so,ab/x.so" reps iters [pytest-targets]
set -uo pipefail
mkdir -p gpurun_out/ab
T=${4:-tests/test_gpu_parity.py}
if [ -n "${PAR_LIB:-}" ]; then export TRITD_LIB=$PWD/$PAR_LIB; fi
timeout -k 10 300 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/par.log 2>&1
rc=$?; tail -2 gpurun_out/ab/par.log; [ $rc -eq 0 ] || exit $rc
unset TRITD_LIB
timeout -k 10 400 python3 tools/ab_lib.py "$1" "$2" "$3"
