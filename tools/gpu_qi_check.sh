set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_qi_model.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/qi_tests.log 2>&1
rc=$?; tail -25 gpurun_out/qi_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/bench4.json 2> gpurun_out/bench4.err || exit $?
cat gpurun_out/bench4.json
