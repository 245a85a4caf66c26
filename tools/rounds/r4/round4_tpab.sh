#!/bin/bash
# Round 4: interleaved primitive A/B over the k_tp variant libraries in ab/,
# then a kernel trace of the primitives for each variant.
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/round4_tpab; mkdir -p $O
timeout -k 10 600 python3 -u tools/ab_prims.py ${LIBS} ${REPS:-3} > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep median $O/ab.log
for l in ${LIBS}; do
  n=$(basename $l .so)
  TRITD_LIB=$PWD/$l timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$n -o run -- \
      python3 -c "import sys; sys.path.insert(0,'.'); import bench; bench.primitives(0, reps=20)" > $O/prof_$n.log 2>&1 || { tail -20 $O/prof_$n.log; exit 1; }
  echo "$n $(grep k_tp $(find $O/prof_$n -name '*kernel_stats.csv' | head -1) | cut -d, -f4)"
done
