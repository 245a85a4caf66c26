#!/bin/bash
# gpurun with a wait for a free GPU slot: retries ONLY while gpurun reports
# that no slot/box was free (exit 3: nothing ran, nothing charged).
#   tools/gpr.sh <timeout-seconds> '<command>'
T=$1; shift
for i in $(seq 1 20); do
    /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
    rc=$?
    [ $rc -ne 3 ] && exit $rc
    echo "[gpr] no slot free (try $i), waiting 90 s" >&2
    sleep 90
done
exit 3
