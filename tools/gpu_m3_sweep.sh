set -uo pipefail
for w in 2048 1024 512 4096; do
  echo "M3_WAVES=$w"
  TRITD_M3_WAVES=$w SHARD_MODES=rccl-sharded timeout -k 10 200 python3 tools/shard_timing.py 8 4 1 2>&1 | grep "P=" || exit 1
done
