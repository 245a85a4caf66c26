set -uo pipefail
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/bench4.json 2> gpurun_out/bench4.err || exit $?
cat gpurun_out/bench4.json
