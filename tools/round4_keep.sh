#!/bin/bash
# Round 4: the store-data keep-alive variants of K5 — correctness of the dense-E
# form at config-3 shapes, then an interleaved config-4 A/B of $AB_LIBS.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for l in ${CHECK_LIBS}; do
  echo "== $l" >> gpurun_out/keep_check.log
  for it in 1 2 3; do
    TRITD_LIB=$l timeout -k 10 200 python -u tools/diag_de3.py 240 320 64 $it 2>&1 | grep differ >> gpurun_out/keep_check.log || exit 1
  done
  DIAG_SHAPES=240x320x64,240x320x300 TRITD_LIB=$l timeout -k 10 300 python -u tools/diag_de.py >> gpurun_out/keep_check.log 2>&1 || exit 1
done
cat gpurun_out/keep_check.log
if [ -n "${AB_LIBS:-}" ]; then
  timeout -k 10 600 python3 -u tools/ab_lib.py ${AB_LIBS} 6 10 > gpurun_out/ab_keep.log 2>&1 || exit $?
  tail -4 gpurun_out/ab_keep.log
fi
