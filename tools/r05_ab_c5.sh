#!/bin/bash
# config-5 K5 pair variants: parity (fp32 tests on each build) and interleaved A/B
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in lean1 lean2; do
  TRITD_LIB=$PWD/ab/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/f32_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 gpurun_out/f32_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
AB_CFG=5 timeout -k 10 600 python3 -u tools/ab_lib.py ab/base.so,ab/lean1.so,ab/lean2.so 4 8 > gpurun_out/ab_c5.log 2>&1 || exit $?
tail -3 gpurun_out/ab_c5.log
timeout -k 10 120 tools/unfold3_probe > gpurun_out/unfold3.log 2>&1 || exit $?
cat gpurun_out/unfold3.log
