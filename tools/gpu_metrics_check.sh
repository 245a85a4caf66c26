# metrics kernels: GPU parity (evaluate, quality_ybz) then the primitive bench
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_metrics.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/metrics_tests.log 2>&1
rc=$?; tail -3 gpurun_out/metrics_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/bench_prims.py > gpurun_out/prims.json 2> gpurun_out/prims.err || exit $?
cat gpurun_out/prims.json
