#!/bin/bash
# Build an experimental variant of libbnpp.so with extra HIP defines into
# bn-pp_amd/lib_<name>/ (host objects shared with the main build).
# usage: tools/build_variant.sh <name> "-DFOO=1 ..."
set -e
cd "$(dirname "$0")/../bn-pp_amd"
name=$1; flags=$2
make -s -j8 lib/libbnpp.so
mkdir -p build_$name lib_$name
rm -f build_$name/*.o
pids=()
for src in csrc/*.hip; do
  f=$(basename $src .hip)
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Icsrc -I../include $flags \
      -c $src -o build_$name/$f.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p || { echo "variant $name: a compile failed"; exit 1; }; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib_$name/libbnpp.so build_$name/*.o \
    build/plan.o build/order.o build/model_io.o build/runtime.o build/capi.o build/bn_api.o -Wl,-soname,libbnpp.so -pthread
echo "built lib_$name"
