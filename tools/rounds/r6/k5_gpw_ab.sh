# Round 6: K5 walking 1 / 2 / 4 ij-tile groups per workgroup (TRITD_K5_GPW), interleaved A/B at
# config 4, with round 5's library as a control, and a bitwise check of the variants
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_gpw; mkdir -p $O
timeout -k 10 300 python3 tools/ab_same.py ab6/base.so,ab6/gpw2.so,ab6/gpw4.so 256 8 12 > $O/same.txt 2>&1
timeout -k 10 600 python3 tools/ab_lib.py ab6/base.so,ab6/gpw2.so,ab6/gpw4.so,ab6/r5.so 4 10 > $O/ab.txt 2>&1
cat $O/same.txt; tail -4 $O/ab.txt
