#!/bin/bash
# PAIR tables in the node classifier: GPU tests (all), then configs 3 / 5c / 6 A/B of the
# out-of-line vs inline fallback.
set -o pipefail
TAG=${1:-pair}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
step() { echo "[$(date +%T)] $*"; }
step tests
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1 || { tail -30 "$O/gpu_tests.log"; exit 1; }
tail -2 "$O/gpu_tests.log"
for lib in libpolicygpu.so libpolicygpu_fbinl.so; do
    for c in 3 5c 6; do
        cnt=""; [ $c = 5c ] && cnt="--counters"
        step sweep $lib config $c
        VPP_AMD_LIB=$R/vpp_amd/$lib timeout -k 10 200 python tools/sweep.py --config ${c%c} --rounds 3 --reps 5 $cnt \
            >> "$O/sweep.jsonl" 2> "$O/sweep.err" || { tail -20 "$O/sweep.err"; exit 1; }
    done
done
python -c "
import json
for l in open('$O/sweep.jsonl'):
    d=json.loads(l); print(d['lib'], d['config'], d['counters'], d['ms'], d['gpps'])
"
step done
