#!/bin/bash
# Refresh the committed evidence under profiles/ (run through gpurun on one
# MI355X; outputs land in gpurun_out/ and are copied into profiles/ locally):
#   two separate PMC passes (FETCH_SIZE, WRITE_SIZE) -> K5 HBM bytes per launch
#   rocprofv3 --kernel-trace --stats of the default bench
#   the default bench line (with cpu_baseline), reading the fresh traffic file
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r01}
ALG=${2:-4831874457}   # K5 algorithmic bytes per launch at 512^3 r=8, derived-Y_O mode (4 dense streams + compact-E slots + W)
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- \
    python3 bench.py --no-cpu --no-e2e --steps 5 --warmup 1 > $O/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- \
    python3 bench.py --no-cpu --no-e2e --steps 5 --warmup 1 > $O/pmc_write.log 2>&1
python3 tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/${TAG}_k5_traffic.json $ALG "k5_fused<64, false" 1:6  # the timed window (warmup 1, steps 5)
cp $O/${TAG}_k5_traffic.json profiles/${TAG}_k5_traffic.json   # read by bench.py below
# MFMA utilisation of K2 (and K5): one SQ/GRBM pass, kernel counters only
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --output-format csv -d $O/pmc_sq -o run -- python3 bench.py --no-cpu --no-e2e --steps 5 --warmup 1 > $O/pmc_sq.log 2>&1
python3 tools/pmc_summary.py --json $O/${TAG}_k2_mfma_util.json $O/pmc_sq "k_m3_cp" "k5_fused<64, false" > $O/${TAG}_mfma_util.txt
cp $O/${TAG}_k2_mfma_util.json profiles/${TAG}_k2_mfma_util.json   # read by bench.py below
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py --no-cpu --no-e2e > $O/stats.log 2>&1
timeout -k 10 400 python3 bench.py > $O/${TAG}_bench_line.json 2> $O/bench.err
cat $O/${TAG}_bench_line.json
# primitive kernels (unfold modes 2/3, soft_threshold, triple_product, evaluate, quality_ybz)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prims_stats -o run -- \
    python3 tools/bench_prims.py > $O/${TAG}_prims.json 2> $O/prims.err
cat $O/${TAG}_prims.json
