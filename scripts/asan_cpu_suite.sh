#!/bin/bash
# The CPU test suite against the ASan/UBSan build of the host C++.
# gcc's runtimes are preloaded into the (uninstrumented) python; leak checking is off
# because the interpreter and torch keep allocations alive at exit.
set -e
cd "$(dirname "$0")/.."
make -s -C generalsparse_amd/csrc san
export GS_LIBRARY=$PWD/generalsparse_amd/libgeneralsparse_san.so
export LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:allocator_may_return_null=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
python -m pytest tests -m "not gpu" -q -p no:xdist -p no:cacheprovider "$@"
