#!/bin/bash
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/diag_c5.py 2 > gpurun_out/diag_c5.log 2>&1
rc=$?; tail -12 gpurun_out/diag_c5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_fullsize.py::test_config5_full_fp32_vs_c_oracle --deselect tests/test_gpu_fullsize.py::test_config4_full_vs_c_oracle --deselect tests/test_gpu_fullsize.py::test_config3_highway_full_vs_c_oracle > gpurun_out/gpu_tests2.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench4.json 2> gpurun_out/bench4.err || exit $?
cut -c1-3000 gpurun_out/bench4.json
