#!/bin/bash
# One GPU-box pass: GPU tests, bench lines, kernel-trace profile and PMC traffic passes.
#   gpurun --timeout 900 -- bash tools/gpu_check.sh TAG [CONFIGS...]
# Writes everything under gpurun_out/TAG/. Stops at the first failing step.
set -o pipefail
TAG=${1:-run}; shift
CONFIGS=${*:-2 4}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
step() { echo "[$(date +%T)] $*"; }

step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1 || { tail -30 "$O/gpu_tests.log"; exit 1; }
tail -2 "$O/gpu_tests.log"

for c in $CONFIGS; do
    step bench config $c
    timeout -k 10 300 python bench.py --config "$c" > "$O/bench_c$c.json" 2> "$O/bench_c$c.err" \
        || { tail -20 "$O/bench_c$c.err"; exit 1; }
    cat "$O/bench_c$c.json"
done

cd /tmp && export TMPDIR=/tmp
for c in $CONFIGS; do
    step rocprof config $c
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c$c" -o run -- \
        python3 "$R/bench.py" --config "$c" --no-cpu --no-check > "$O/prof_c$c.log" 2>&1 \
        || { tail -20 "$O/prof_c$c.log"; exit 1; }
    for ctr in FETCH_SIZE WRITE_SIZE; do
        step pmc $ctr config $c
        timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$O/pmc_${ctr}_c$c" -o run -- \
            python3 "$R/bench.py" --config "$c" --no-cpu --no-check --steps 3 --warmup 1 > "$O/pmc_${ctr}_c$c.log" 2>&1 \
            || { tail -20 "$O/pmc_${ctr}_c$c.log"; exit 1; }
    done
done
step done
