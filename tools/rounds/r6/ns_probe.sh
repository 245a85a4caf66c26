#!/bin/bash
# Round 6: where the sharded update_B solve (k_solve_ns<64>, ~18 us per P = 8 iteration) spends its
# time — timing-only probe libraries: 1 = no finish of the previous iteration, 2 = one Newton update,
# 3 = always the sweep; P = 8 shard timing under a kernel trace for each.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_ns; mkdir -p $O
for l in base ns1 ns2 ns3; do
  TRITD_LIB=$PWD/ab6/$l.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$l -o run -- python3 tools/shard_timing.py 8 > $O/$l.log 2>&1
done
python3 - <<'PY' > $O/summary.txt
import csv, glob, statistics as st
for l in ["base", "ns1", "ns2", "ns3"]:
    f = glob.glob("gpurun_out/r6_ns/%s/**/run_kernel_trace.csv" % l, recursive=True)[0]
    r = list(csv.DictReader(open(f)))
    d = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3 for x in r if "k_solve_ns" in x["Kernel_Name"]]
    print(l, "k_solve_ns n=%d median %.2f us, last 50 median %.2f" % (len(d), st.median(d), st.median(d[-50:])))
PY
cat $O/summary.txt
grep -h "P=8" $O/*.log
echo done
