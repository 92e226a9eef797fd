#!/bin/bash
# GPU test pass: every -m gpu test (or the given pytest args), one process, per-test timeout.
#   gpurun --timeout 900 -- bash tools/gpu_tests.sh TAG [pytest args...]
set -o pipefail
TAG=${1:-tests}; shift
O=$(pwd)/gpurun_out/$TAG
mkdir -p "$O"
[ $# -gt 0 ] || set -- tests
echo "[$(date +%T)] pytest -m gpu $*"
timeout -k 10 840 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" "$O/gpu_tests.log" | tail -60
[ $rc -eq 0 ] || tail -60 "$O/gpu_tests.log"
exit $rc
