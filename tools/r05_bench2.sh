#!/bin/bash
# bench.py's N > 1 path on one GPU: two ranks, gloo + libtritd's host all-reduce transport
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --steps 5 --warmup 2 --comm host --no-e2e > gpurun_out/bench_n2host.json 2> gpurun_out/bench_n2host.err || exit $?
cut -c1-700 gpurun_out/bench_n2host.json
timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --no-cpu > gpurun_out/bench4b.json 2> gpurun_out/bench4b.err || exit $?
cut -c1-400 gpurun_out/bench4b.json
timeout -k 10 300 python3 bench.py --config 5 --steps 10 --warmup 3 --no-cpu --no-e2e > gpurun_out/bench5b.json 2> gpurun_out/bench5b.err || exit $?
cut -c1-400 gpurun_out/bench5b.json
