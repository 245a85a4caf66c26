#!/bin/bash
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_dist_host.py tests/test_gpu_flags.py tests/test_gpu_metrics.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/ts.log 2>&1
rc=$?; echo "tests: $(tail -1 gpurun_out/ts.log)"; [ $rc -eq 0 ] || exit $rc
for c in 2 4; do
  timeout -k 10 300 python3 bench.py --config $c --steps 40 --warmup 25 --no-cpu --no-e2e > gpurun_out/bench_ts_c$c.json 2> gpurun_out/bench_ts_c$c.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/bench_ts_c$c.json'));print($c, round(d['value'],1), d['kernel_ms'], round(d['roofline']['frac'],3), d['rre_final'], d['k_final'])"
done
