#!/bin/bash
# Round 4: K5 variant libraries — a GPU test subset on each of $CHECK_LIBS
# (TRITD_LIB), then an interleaved config-4 A/B of $AB_LIBS.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="${TESTS:-tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_determinism.py}"
for l in ${CHECK_LIBS:-}; do
  n=$(basename $l .so)
  TRITD_LIB=$l timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/var_tests_$n.log 2>&1
  rc=$?; echo "$l: $(tail -1 gpurun_out/var_tests_$n.log)"; [ $rc -eq 0 ] || exit $rc
done
if [ -n "${AB_LIBS:-}" ]; then
  timeout -k 10 600 python3 -u tools/ab_lib.py ${AB_LIBS} ${AB_REPS:-6} 10 > gpurun_out/ab_var.log 2>&1 || exit $?
  tail -4 gpurun_out/ab_var.log
fi
