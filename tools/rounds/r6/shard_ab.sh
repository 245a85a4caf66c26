# Round 6: P = 8 shard timing, this build against round 5's library (TRITD_LIB), interleaved
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_shard_ab; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 200 python3 tools/shard_timing.py 8 >> $O/shard_new.txt 2>&1
  TRITD_LIB=$PWD/ab6/r5.so timeout -k 10 200 python3 tools/shard_timing.py 8 >> $O/shard_r5.txt 2>&1
done
grep "P=8" $O/shard_new.txt $O/shard_r5.txt
