#!/bin/bash
# Link a library variant with the listed sources rebuilt under extra flags (A/B measurement only).
# Usage: bash scripts/build_variant2.sh NAME "-DFOO=1 ..." src1.hip [src2.hip ...]   -> var/NAME.so
set -e
cd "$(dirname "$0")/../medical-vision-textural-bias_amd/csrc"
make -s -j8 >/dev/null
name=$1; flags=$2; shift 2
mkdir -p build/var_$name ../../var
extra=""
objs=$(ls build/*.o)
for src in "$@"; do
  b=$(basename $src .hip)
  nof="-fno-slp-vectorize"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -I. -Wall -Wno-unused-function \
    -Wno-unknown-pragmas $nof $flags -c $src -o build/var_$name/$b.o
  objs=$(echo "$objs" | grep -v "/$b.o$")
  extra="$extra build/var_$name/$b.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs $extra -o ../../var/$name.so
echo "var/$name.so"
