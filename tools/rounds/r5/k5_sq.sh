#!/bin/bash
# Round 5: config-4 K5 (k5_fused<64,false,false>) SQ issue/wait breakdown in
# three PMC passes (kernel counters only), plus the P = 8 shard timing under
# a kernel trace.  Summaries: gpurun_out/r5_k5sq/*.txt
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_k5sq; mkdir -p $O
B="python3 bench.py --no-cpu --no-e2e --no-prims --steps 5 --warmup 1"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS \
    --output-format csv -d $O/p1 -o run -- $B > $O/p1.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_WAVES \
    --output-format csv -d $O/p2 -o run -- $B > $O/p2.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $O/p3 -o run -- $B > $O/p3.log 2>&1 || exit $?
python3 tools/pmc_summary.py $O "k5_fused<64, false, false" "k_m3_cp" > $O/k5_sq.txt
cat $O/k5_sq.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/shard -o run -- \
    python3 tools/shard_timing.py 8 > $O/shard8.txt 2>&1 || exit $?
cat $O/shard8.txt
