#!/bin/bash
# rocprofv3 --kernel-trace --stats of the config-2 and config-3 bench runs
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for c in 2 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c${c}stats -o run -- \
      python3 bench.py --config $c --no-cpu --no-e2e --steps 40 --warmup 25 > gpurun_out/c${c}stats.log 2>&1 || exit $?
  echo "config $c: $(grep '^{' gpurun_out/c${c}stats.log | head -1 | cut -c1-200)"
done
