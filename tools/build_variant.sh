#!/bin/bash
# Build an experimental variant of libbnpp.so with extra defines into
# bn-pp_amd/lib_<name>/ (HIP and host sources), e.g. -DBNPP_TUNING_KNOBS for
# the planner's A/B knobs or -DBNPP_STREAM_U=16 for a kernel constant.
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
  extra=""
  case $f in k_generic2_*) extra="-mllvm -sink-common-insts=false";; esac     # as the Makefile
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Icsrc -I../include $flags $extra \
      -c $src -o build_$name/$f.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p || { echo "variant $name: a compile failed"; exit 1; }; done
# host sources with the same defines (-DBNPP_TUNING_KNOBS: the planner's tuning knobs, plan.hpp)
pids=()
for src in csrc/plan.cpp csrc/order.cpp csrc/model_io.cpp csrc/runtime.cpp csrc/capi.cpp csrc/bn_api.cpp; do
  f=$(basename $src .cpp)
  g++ -O3 -std=c++17 -fPIC -Wall -Wextra -ffp-contract=off -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Icsrc -I../include \
      $flags -c $src -o build_$name/host_$f.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p || { echo "variant $name: a compile failed"; exit 1; }; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib_$name/libbnpp.so build_$name/*.o \
    -Wl,-soname,libbnpp.so -pthread
echo "built lib_$name"
