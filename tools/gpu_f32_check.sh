set -uo pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/f32_tests.log 2>&1
rc=$?; tail -2 gpurun_out/f32_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --config 5 --steps 10 --warmup 3 --no-cpu > gpurun_out/bench5.json 2> gpurun_out/bench5.err || exit $?
cat gpurun_out/bench5.json
