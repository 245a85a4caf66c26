#!/bin/bash
# multi-workgroup solve: microbench + config-5 one-shot diagnosis + full-size
# config-5 test + config-5 bench line
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rp in "128 128" "128 121" "256 256" "256 225"; do
  timeout -k 10 60 tools/solve_mw_bench $rp >> gpurun_out/solve_mw.log 2>&1 || exit $?
  TRITD_SOLVE=big timeout -k 10 60 tools/solve_mw_bench $rp >> gpurun_out/solve_mw.log 2>&1 || exit $?
done
cat gpurun_out/solve_mw.log
timeout -k 10 400 python3 -u tools/diag_c5.py 2 > gpurun_out/diag_c5.log 2>&1
rc=$?; tail -8 gpurun_out/diag_c5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_f32.py -m gpu -x -v -s --timeout 600 --timeout-method thread -p no:cacheprovider -k "config5 or large_rank or f32_vs" > gpurun_out/gpu_c5.log 2>&1
rc=$?; tail -12 gpurun_out/gpu_c5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --config 5 --no-cpu --steps 10 --warmup 3 > gpurun_out/bench5.json 2> gpurun_out/bench5.err || exit $?
cut -c1-1500 gpurun_out/bench5.json
