#!/bin/bash
# dense-E K5 mode: parity (forced from the start on the goldens, automatic on the
# video-like full-size config 3) and the config 2 / 3 / 4 bench lines
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TRITD_DENSE_E=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/de_forced.log 2>&1
rc=$?; echo "forced: $(tail -1 gpurun_out/de_forced.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider -k config3 > gpurun_out/de_c3.log 2>&1
rc=$?; echo "config3: $(tail -1 gpurun_out/de_c3.log)"; [ $rc -eq 0 ] || exit $rc
for c in 3 2 4; do
  timeout -k 10 300 python3 bench.py --config $c --steps 40 --warmup 25 --no-cpu > gpurun_out/bench_de_c$c.json 2> gpurun_out/bench_de_c$c.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/bench_de_c$c.json'));print($c, round(d['value'],1), d['kernel_ms'], d['roofline']['dense_streams'], round(d['roofline']['frac'],3), d['rre_final'], d['k_final'])"
done
