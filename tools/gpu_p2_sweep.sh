set -uo pipefail
for cfg in "0 256" "1 256" "0 4352" "0 33024" "1 4352"; do
  set -- $cfg
  echo "ROT=$1 STAGGER=$2"
  for P in 2 1; do
    TRITD_ROT=$1 TRITD_STAGGER=$2 SHARD_MODES=rccl-sharded timeout -k 10 120 python3 tools/shard_timing.py $P 2>&1 | grep "P=" || exit 1
  done
done
