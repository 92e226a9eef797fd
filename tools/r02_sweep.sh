#!/bin/bash
# Rule-count sweep (bench.py --rules N on config 2's gen-policy shape, and config 7: the whole
# gen-policy.py policy through the configurator), driver bench settings, one line each.
#   gpurun --timeout 900 -- bash tools/r02_sweep.sh TAG [pytest first: 1]
set -o pipefail
TAG=${1:-sweep}; TESTS=${2:-1}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
step() { echo "[$(date +%T)] $*"; }
if [ "$TESTS" = 1 ]; then
step tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1 || { tail -30 "$O/gpu_tests.log"; exit 1; }
tail -2 "$O/gpu_tests.log"
fi
for n in 1000 10000 100000; do
    step rules $n
    timeout -k 10 300 python bench.py --config 2 --rules $n > "$O/bench_rules$n.json" 2> "$O/bench_rules$n.err" \
        || { tail -20 "$O/bench_rules$n.err"; exit 1; }
    cut -c1-200 "$O/bench_rules$n.json"; grep -o '"roofline": {[^}]*}' "$O/bench_rules$n.json"
done
step config 7
timeout -k 10 400 python bench.py --config 7 > "$O/bench_c7.json" 2> "$O/bench_c7.err" || { tail -20 "$O/bench_c7.err"; exit 1; }
cut -c1-200 "$O/bench_c7.json"; grep -o '"roofline": {[^}]*}' "$O/bench_c7.json"
step done
