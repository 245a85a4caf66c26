#!/bin/bash
# Round 4: kernel-trace statistics of the bench at configs 2, 3 and 5 (one
# MI355X), written under gpurun_out/round4_small.
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/round4_small
mkdir -p $O
for c in ${CONFIGS:-2 3 5}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c$c -o run -- \
      python3 bench.py --config $c --no-cpu --no-e2e --no-prims > $O/c$c.json 2> $O/c$c.err || exit $?
  cut -c1-160 $O/c$c.json
done
