#!/bin/bash
# Round 5 evidence on one MI355X (outputs in gpurun_out/r5_ev, copied into
# profiles/round5 by hand): K5 PMC traffic (separate FETCH_SIZE / WRITE_SIZE
# passes) and MFMA utilisation for config 4 and config 5, rocprofv3
# --kernel-trace --stats of the default bench, the P = 8 shard trace.
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_ev; mkdir -p $O
B4="python3 bench.py --no-cpu --no-e2e --no-prims --no-c5 --steps 5 --warmup 1"
B5="python3 bench.py --config 5 --no-cpu --no-e2e --no-prims --no-c5 --steps 3 --warmup 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B4 > $O/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B4 > $O/pmc_write.log 2>&1 || exit $?
python3 tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/k5_traffic.json 4831874457 "k5_fused<64, false" 1:6 > $O/k5_traffic.txt 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --output-format csv -d $O/pmc_sq -o run -- $B4 > $O/pmc_sq.log 2>&1 || exit $?
python3 tools/pmc_summary.py --json $O/k2_mfma_util.json $O/pmc_sq "k_m3_cp" "k5_fused<64, false" > $O/mfma_util.txt 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c5_pmc_fetch -o run -- $B5 > $O/c5_pmc_fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c5_pmc_write -o run -- $B5 > $O/c5_pmc_write.log 2>&1 || exit $?
python3 tools/pmc_traffic.py $O/c5_pmc_fetch $O/c5_pmc_write $O/c5_k5_traffic.json 32212254720 "k5_f32s<256>" 1:4 > $O/c5_k5_traffic.txt 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --output-format csv -d $O/c5_pmc_sq -o run -- $B5 > $O/c5_pmc_sq.log 2>&1 || exit $?
python3 tools/pmc_summary.py --json $O/c5_k2_mfma_util.json $O/c5_pmc_sq "k_m3_32<256" "k5_f32s<256>" > $O/c5_mfma_util.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py --no-cpu --no-e2e --no-c5 > $O/stats.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/shard -o run -- \
    python3 tools/shard_timing.py 8 > $O/shard.txt 2>&1 || exit $?
python3 tools/trace_iter.py $O/shard/run_kernel_trace.csv 3 "k5_fused<" > $O/shard_iter.txt 2>&1
timeout -k 10 200 python3 tools/shard_timing.py 4 2 >> $O/shard.txt 2>&1
