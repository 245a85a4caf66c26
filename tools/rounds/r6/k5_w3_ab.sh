# Round 6: is three waves per SIMD worth it for K5?  The one instance that fits 168 VGPRs and
# 53 KB of LDS at TRITD_K5_WPE=3 is the dense-E RP = 32 one: 512^3 r = 5 with E forced dense,
# this build (2 waves/SIMD) vs the WPE=3 build, interleaved; plus the compact-E r = 8 instance
# (which the WPE=3 build cannot fit: it falls back to fewer waves) as a control.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_w3; mkdir -p $O
AB_R=5 TRITD_DENSE_E=1 timeout -k 10 500 python3 tools/ab_lib.py ab6/base.so,ab6/w3.so 4 10 > $O/ab_r5_dense.txt 2>&1
AB_R=8 timeout -k 10 500 python3 tools/ab_lib.py ab6/base.so,ab6/w3.so 3 10 > $O/ab_r8.txt 2>&1
tail -n 2 $O/ab_r5_dense.txt $O/ab_r8.txt
