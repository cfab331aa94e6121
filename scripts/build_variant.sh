#!/bin/bash
# Link a library variant with some kernel sources rebuilt under extra flags (A/B measurement only).
# Usage: bash scripts/build_variant.sh NAME "-DFOO=1 ..." ["kern_band kern_slab_ct ..."]  -> var/NAME.so
# (sources default to kern_band; each is rebuilt with -fno-slp-vectorize, as the Makefile does)
set -e
cd "$(dirname "$0")/../medical-vision-textural-bias_amd/csrc"
make -s -j8 >/dev/null
srcs=${3:-kern_band}
mkdir -p build/var_$1 ../../var
objs=$(ls build/*.o)
for s in $srcs; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -I. -Wall -Wno-unused-function \
    -Wno-unknown-pragmas -fno-slp-vectorize $2 -c $s.hip -o build/var_$1/$s.o
  objs=$(echo "$objs" | grep -v "^build/$s.o$")
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs build/var_$1/*.o -o ../../var/$1.so
echo "var/$1.so"
