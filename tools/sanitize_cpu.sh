#!/bin/bash
# Host-code sanitizer run: the CPU test suite against
# build-san/libbwtmi_san.so (ASan + UBSan on every host path: loader,
# post-processing folds, writers, C ABI; the device code is not instrumented
# and no GPU is used).  Python itself is not instrumented, so the ASan runtime
# is preloaded and leak checking is off (the interpreter's own allocations).
set -o pipefail
cd "$(dirname "$0")/.."
make -s -C bwt-algorithm_amd san
RT=$(/opt/rocm/llvm/bin/clang++ -print-file-name=libclang_rt.asan-x86_64.so)
export BWTMI_LIB=$PWD/bwt-algorithm_amd/build-san/libbwtmi_san.so
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:verify_asan_link_order=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD=$RT timeout -k 10 ${SAN_TIMEOUT:-2400} python -m pytest tests -m "not gpu" -x -q -p no:cacheprovider "$@"
