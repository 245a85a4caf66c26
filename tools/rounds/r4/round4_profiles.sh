#!/bin/bash
# Round 4 evidence, written under gpurun_out/round4 (copied into profiles/round4 by hand):
#   optional pytest subset ($TESTS), then two separate PMC passes (FETCH_SIZE,
#   WRITE_SIZE) -> K5 HBM bytes per launch; one SQ/GRBM pass -> MFMA
#   utilisation of K2 / K5; rocprofv3 --kernel-trace --stats of the bench;
#   the full bench line; the primitives under --stats.
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/round4
mkdir -p $O
ALG=4831874457   # K5 algorithmic bytes per launch at 512^3 r=8 (4 dense streams + compact-E slots + W)
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
  rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
B="python3 bench.py --no-cpu --no-e2e --no-prims --steps 5 --warmup 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B > $O/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B > $O/pmc_write.log 2>&1 || exit $?
python3 tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/k5_traffic.json $ALG "k5_fused<64, false" 1:6 || exit $?
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --output-format csv -d $O/pmc_sq -o run -- $B > $O/pmc_sq.log 2>&1 || exit $?
python3 tools/pmc_summary.py --json $O/k2_mfma_util.json $O/pmc_sq "k_m3_cp" "k5_fused<64, false" > $O/mfma_util.txt || exit $?
# the bench line below cites the newest profiles/round*/ PMC files: this run's
mkdir -p profiles/round4 && cp $O/k5_traffic.json $O/k2_mfma_util.json profiles/round4/
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py --no-cpu --no-e2e --no-prims > $O/stats.log 2>&1 || exit $?
timeout -k 10 500 python3 bench.py > $O/bench_line.json 2> $O/bench.err || exit $?
cut -c1-400 $O/bench_line.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prims_stats -o run -- \
    python3 tools/bench_prims.py > $O/prims.json 2> $O/prims.err || exit $?
find $O/stats $O/prims_stats -name "*kernel_stats.csv" | head -3
if [ -n "${SMALL:-}" ]; then
  timeout -k 10 300 python3 bench.py --config 2 --no-e2e --no-prims > $O/c2_bench_line.json 2> $O/c2.err || exit $?
  timeout -k 10 300 python3 bench.py --config 3 --no-e2e --no-prims > $O/c3_bench_line.json 2> $O/c3.err || exit $?
  timeout -k 10 400 python3 bench.py --config 5 --no-e2e --no-prims --no-cpu > $O/c5_bench_line.json 2> $O/c5.err || exit $?
  cut -c1-200 $O/c2_bench_line.json $O/c3_bench_line.json $O/c5_bench_line.json
fi
