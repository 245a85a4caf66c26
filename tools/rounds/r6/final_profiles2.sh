# (second pass, final build: the same evidence plus the default bench line on the same box)
# Round 6 evidence ($O/): K5 HBM bytes per launch from two separate PMC passes (config 4
# and config 5), K2 / K5 MFMA utilisation (SQ pass), rocprofv3 --kernel-trace --stats of the bench,
# the default bench line, smoke().  Run through gpurun on one MI355X.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_final2; mkdir -p $O
B4="python3 bench.py --no-cpu --no-e2e --no-prims --no-c5 --steps 5 --warmup 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B4 > $O/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B4 > $O/pmc_write.log 2>&1
python3 tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/k5_traffic.json 4831874457 "k5_fused<64, false" 1:6
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --output-format csv -d $O/pmc_sq -o run -- $B4 > $O/pmc_sq.log 2>&1
python3 tools/pmc_summary.py --json $O/k2_mfma_util.json $O/pmc_sq "k_m3_cp" "k5_fused<64, false" > $O/mfma_util.txt
B5="python3 bench.py --config 5 --no-cpu --no-e2e --no-prims --steps 3 --warmup 1"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c5_fetch -o run -- $B5 > $O/c5_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c5_write -o run -- $B5 > $O/c5_write.log 2>&1
python3 tools/pmc_traffic.py $O/c5_fetch $O/c5_write $O/c5_k5_traffic.json 32212254720 "k5_f32s<256>" 1:4
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --output-format csv -d $O/c5_sq -o run -- $B5 > $O/c5_sq.log 2>&1
python3 tools/pmc_summary.py --json $O/c5_k2_mfma_util.json $O/c5_sq "k_m3_32<256" "k5_f32s<256>" > $O/c5_mfma_util.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py --no-cpu --no-e2e --no-c5 > $O/stats.log 2>&1
cp $O/stats/run_kernel_stats.csv $O/bench_kernel_stats.csv
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log.txt 2>&1
timeout -k 10 600 python3 bench.py > $O/bench_line.json 2> $O/bench.err
echo done
