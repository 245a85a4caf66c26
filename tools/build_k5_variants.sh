#!/bin/bash
# Build libtritd variants that differ only in the -D flags of the kernel files (k_*.hip), into ab6/<name>.so
#   bash tools/build_k5_variants.sh name1="-DK5_EXP=1" name2="-DFOO=2" ...
set -e
cd "$(dirname "$0")/../triple-tensor-decomposition-with-admm_amd/csrc"
make -j8 >/dev/null
mkdir -p ../../ab6
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  rm -rf build_$name; cp -r build build_$name; rm -f build_$name/k_*.o build_$name/solver.o build_$name/api.o
  make OBJDIR=build_$name OUT=../../ab6/$name.so EXTRA="$flags" >/dev/null &
done
wait
cp ../tritd/libtritd.so ../../ab6/base.so
ls -la ../../ab6
