#!/bin/bash
# Round 4: k_tp variant — triple-product tests on $LIB, an interleaved
# primitive A/B against ab/prev.so, and a kernel trace of the primitives.
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/round4_tp; mkdir -p $O
LIB=${LIB:-ab/tp4.so}
TRITD_LIB=$PWD/$LIB timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_flags.py} \
    -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python3 -u tools/ab_prims.py ab/prev.so $LIB ${REPS:-4} > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep median $O/ab.log
TRITD_LIB=$PWD/$LIB timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 -c "import sys; sys.path.insert(0,'.'); import bench; bench.primitives(0, reps=20)" > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs cut -c1-200
