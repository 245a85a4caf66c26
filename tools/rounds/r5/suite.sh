#!/bin/bash
# Round 5: full GPU suite, smoke, default bench line (one box, one call)
O=gpurun_out/${1:-r5_suite}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench.txt 2>&1
