#!/bin/bash
# The host-threading tests (tests/test_threads_host.py: contexts driven from several OS threads at
# once, and the counter snapshots read by gauge threads while replaced, test_stats_host.py)
# once, the way cgo callers may) against the TSan build of the host C++ layer
# (make -C vpp_amd/csrc tsan). Any data-race report fails the run (halt_on_error).
#   bash tools/tsan_tests.sh [pytest args]
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
make -s -j8 -C "$R/vpp_amd/csrc" tsan || exit 1
export VPP_AMD_LIB=$R/vpp_amd/libpolicygpu_tsan.so
export LD_PRELOAD=$(gcc -print-file-name=libtsan.so)
export TSAN_OPTIONS="halt_on_error=1 exitcode=66 report_signal_unsafe=0 ignore_noninstrumented_modules=1 ${TSAN_LOG:+log_path=$TSAN_LOG}"
cd "$R" && python -m pytest tests/test_threads_host.py tests/test_stats_host.py::test_snapshot_readers_race_a_writer \
    tests/test_stats_host.py::test_layout_generation_polled_during_recompiles \
    tests/test_stats_host.py::test_counts_survive_a_commit_that_changes_another_acl -x -q -s -p no:cacheprovider ${*}
