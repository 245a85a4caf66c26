set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_c5ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_bench_launch.py -k torchrun > $O/torchrun.log 2>&1
AB_CFG=5 AB_WARM=5 timeout -k 10 500 python -u tools/ab_lib.py ab6/base.so,ab6/xcd0.so 3 10 > $O/ab.txt 2>&1
B="python3 bench.py --config 5 --no-cpu --no-e2e --no-prims --steps 3 --warmup 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B > $O/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B > $O/pmc_write.log 2>&1
python3 tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/c5_k5_traffic.json 32212254720 "k5_f32s<256>" 1:4 > $O/traffic.txt 2>&1
echo done
