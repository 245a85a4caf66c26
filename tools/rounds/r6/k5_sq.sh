#!/bin/bash
# Round 6, last build: the SQ issue / wait breakdown of round 5's tools/rounds/r5/k5_sq.sh for config-4
# K5 and K2, and the same passes for config 5's K5 (k5_f32s) and K2 (k_m3_32) — kernel counters only,
# one pass per counter group.  Summaries: gpurun_out/r6_k5sq/{c4,c5}_sq.txt
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_k5sq; mkdir -p $O
B4="python3 bench.py --no-cpu --no-e2e --no-prims --no-c5 --steps 5 --warmup 1"
B5="python3 bench.py --config 5 --no-cpu --no-e2e --no-prims --steps 3 --warmup 1"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_WAVES"
P3="SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d $O/c4p$i -o run -- $B4 > $O/c4p$i.log 2>&1 || exit $?
done
mkdir -p $O/c4 && mv $O/c4p1 $O/c4/p1 && mv $O/c4p2 $O/c4/p2 && mv $O/c4p3 $O/c4/p3
python3 tools/pmc_summary.py $O/c4 "k5_fused<64, false, false" "k_m3_cp" > $O/c4_sq.txt
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d $O/c5p$i -o run -- $B5 > $O/c5p$i.log 2>&1 || exit $?
done
mkdir -p $O/c5 && mv $O/c5p1 $O/c5/p1 && mv $O/c5p2 $O/c5/p2 && mv $O/c5p3 $O/c5/p3
python3 tools/pmc_summary.py $O/c5 "k5_f32s<256>" "k_m3_32<256" > $O/c5_sq.txt
echo done
