#!/bin/bash
# Host-code sanitizer runs of the CPU test suite; the device code
# is not instrumented and no GPU is used.  Python itself is not instrumented,
# so the sanitizer runtime is preloaded (ahead of anything already preloaded).
#   tools/sanitize_cpu.sh [asan] [pytest args]   ASan + UBSan: build-san/libbwtmi_san.so
#                                                (leak checking off: the interpreter's own allocations)
#   tools/sanitize_cpu.sh tsan [pytest args]     ThreadSanitizer: build-tsan/libbwtmi_tsan.so (pool
#                                                hand-off, reaper, parallel record construction)
set -o pipefail
cd "$(dirname "$0")/.."
MODE=asan
if [ "$1" = asan ] || [ "$1" = tsan ]; then MODE=$1; shift; fi
if [ $MODE = asan ]; then
  make -s -C bwt-algorithm_amd san || exit 1
  RT=$(/opt/rocm/llvm/bin/clang++ -print-file-name=libclang_rt.asan-x86_64.so)
  export BWTMI_LIB=$PWD/bwt-algorithm_amd/build-san/libbwtmi_san.so
  export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:verify_asan_link_order=0
  export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
else
  make -s -j8 -C bwt-algorithm_amd tsan || exit 1
  RT=$(/opt/rocm/llvm/bin/clang++ -print-file-name=libclang_rt.tsan-x86_64.so)
  export BWTMI_LIB=$PWD/bwt-algorithm_amd/build-tsan/libbwtmi_tsan.so
  export TSAN_OPTIONS=halt_on_error=1:abort_on_error=1:report_signal_unsafe=0:second_deadlock_stack=1:suppressions=$PWD/tools/tsan.supp:${TSAN_EXTRA:-}
fi
LD_PRELOAD=$RT${LD_PRELOAD:+:$LD_PRELOAD} timeout -k 10 ${SAN_TIMEOUT:-2400} python -m pytest tests -m "not gpu" -x -q -p no:cacheprovider "$@"
