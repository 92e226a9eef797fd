#!/bin/bash
# The CPU test suite against the ASan + UBSan build of the host C++ layer
# (make -C vpp_amd/csrc asan). Leak checking is off: the Python interpreter's own allocations
# would drown it. Any ASan / UBSan report aborts the test process.
#   bash tools/asan_tests.sh [pytest args]
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
make -s -j8 -C "$R/vpp_amd/csrc" asan || exit 1
export VPP_AMD_LIB=$R/vpp_amd/libpolicygpu_asan.so
export LD_PRELOAD=$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
cd "$R" && python -m pytest tests -m "not gpu" -x -q -p no:cacheprovider ${*:---deselect tests/test_multirank.py}
