#!/bin/bash
# Link a library variant with kern_band.hip rebuilt under extra flags (A/B measurement only).
# Usage: bash scripts/build_variant.sh NAME "-DFOO=1 ..."   -> var/NAME.so
set -e
cd "$(dirname "$0")/../medical-vision-textural-bias_amd/csrc"
make -s -j8 >/dev/null
mkdir -p build/var_$1 ../../var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -I. -Wall -Wno-unused-function \
  -Wno-unknown-pragmas -fno-slp-vectorize $2 -c kern_band.hip -o build/var_$1/kern_band.o
objs=$(ls build/*.o | grep -v '/kern_band.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs build/var_$1/kern_band.o -o ../../var/$1.so
echo "var/$1.so"
