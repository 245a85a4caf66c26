#!/bin/bash
# Config-5 evidence (2048x2048x256 r=16 fp32, bench.py --config 5) under
# profiles/: PMC traffic of the fused update (separate FETCH_SIZE /
# WRITE_SIZE passes), rocprofv3 --kernel-trace --stats, and the bench line
# with its one-iteration CPU sample.  Run through gpurun on one MI355X.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r01}
ALG=${2:-32212254720}   # K5 algorithmic bytes per launch at config 5 without dense E tiles
O=gpurun_out/${TAG}_c5
mkdir -p $O
B="python3 bench.py --config 5 --no-cpu --no-e2e --steps 3 --warmup 1"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- \
    $B > $O/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- \
    $B > $O/pmc_write.log 2>&1
python3 tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/${TAG}_c5_k5_traffic.json $ALG "k5_f32s<256>" 1:4  # timed window (warmup 1, steps 3): E densifies later
cp $O/${TAG}_c5_k5_traffic.json profiles/${TAG}_c5_k5_traffic.json
# MFMA utilisation of K2 (k_m3_32) and K5: one SQ/GRBM pass, kernel counters only
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --output-format csv -d $O/pmc_sq -o run -- $B > $O/pmc_sq.log 2>&1
python3 tools/pmc_summary.py --json $O/${TAG}_c5_k2_mfma_util.json $O/pmc_sq "k_m3_32<256" "k5_f32s<256>" > $O/${TAG}_c5_mfma_util.txt
cp $O/${TAG}_c5_k2_mfma_util.json profiles/${TAG}_c5_k2_mfma_util.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py --config 5 --no-cpu --no-e2e --steps 10 --warmup 3 > $O/stats.log 2>&1
timeout -k 10 500 python3 bench.py --config 5 --steps 10 --warmup 3 > $O/${TAG}_c5_bench_line.json 2> $O/bench.err
cat $O/${TAG}_c5_bench_line.json
