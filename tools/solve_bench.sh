#!/bin/bash
# build the k_solve variants of tools/solve_bench.hip (run them on the GPU box)
set -e
cd "$(dirname "$0")"
I="-I../include -I../triple-tensor-decomposition-with-admm_amd/csrc"
F="-O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950"
for rows in 4 8 16; do
  for rcp in 0; do
    D="-DSOLVE_ROWS_OVERRIDE=$rows"; [ $rcp = 1 ] && D="$D -DSOLVE_RCP"
    /opt/rocm/bin/hipcc $F $I $D -DVARIANT="\"rows=$rows rcp=$rcp\"" solve_bench.hip -o solve_bench_${rows}_${rcp} &
  done
done
wait
