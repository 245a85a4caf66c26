set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_m2probe; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/a -o run -- python3 bench.py --no-cpu --no-e2e --no-prims --no-c5 --steps 20 --warmup 2 > $O/a.log 2>&1
TRITD_XB=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b -o run -- python3 bench.py --no-cpu --no-e2e --no-prims --no-c5 --steps 20 --warmup 2 > $O/b.log 2>&1
echo done
