#!/bin/bash
# Host code under ASan + UBSan (CPU, build container): build
# bn-pp_amd/lib_san/libbnpp.so and run the host tests (planner, ABI
# validation, UAI loader, ordering, bucket-tree and chain planning, the C++
# mirror's compile) against it.  Leak checking is off (the Python interpreter's
# own allocations are not ours to judge); any ASan/UBSan report fails the run.
set -eo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
make -C "$R/bn-pp_amd" sanitize -j8 > /dev/null
export BNPP_LIB="$R/bn-pp_amd/lib_san/libbnpp.so"
export LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
cd "$R"
python3 -m pytest tests/test_host.py -x -q -m "not gpu" -p no:cacheprovider "$@"
