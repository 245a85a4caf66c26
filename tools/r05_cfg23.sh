#!/bin/bash
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for c in 3 2; do
  timeout -k 10 300 python3 bench.py --config $c --steps 40 --warmup 5 > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err
  rc=$?; cut -c1-1200 gpurun_out/bench_c$c.json; tail -2 gpurun_out/bench_c$c.err; [ $rc -eq 0 ] || exit $rc
done
