#!/bin/bash
# Config-4 evidence refresh (tools/refresh_profiles.sh r05) plus the config-2/3
# bench lines, on the final build
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/refresh_profiles.sh r05 > gpurun_out/refresh_c4.log 2>&1 || exit $?
tail -3 gpurun_out/refresh_c4.log | cut -c1-300
for c in 2 3; do
  timeout -k 10 300 python3 bench.py --config $c --steps 40 --warmup 25 --no-e2e > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/bench_c$c.json'));print($c, round(d['value'],1), d['kernel_ms'], round(d['roofline']['frac'],3), d['rre_final'], d['k_final'])"
done
