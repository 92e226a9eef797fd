#!/bin/bash
# Node kernels (configs 3 / 5 / 6): A/B of measurement and chunk builds, and the rule-count sweep.
set -o pipefail
TAG=${1:-abnode}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
step() { echo "[$(date +%T)] $*"; }
for r in 1 2; do
for lib in libpolicygpu.so libpolicygpu_nofb.so libpolicygpu_nofbq2.so libpolicygpu_q2.so; do
    for c in 3 5; do
        cnt=""; [ $c = 5 ] && cnt="--counters"
        step sweep $lib config $c
        VPP_AMD_LIB=$R/vpp_amd/$lib timeout -k 10 200 python tools/sweep.py --config $c --rounds 3 --reps 5 $cnt \
            >> "$O/sweep.jsonl" 2> "$O/sweep.err" || { tail -20 "$O/sweep.err"; exit 1; }
    done
done
done
python -c "
import json
for l in open('$O/sweep.jsonl'):
    d=json.loads(l); print(d['lib'], d['config'], d['counters'], d['ms'], d['gpps'])
"
for n in 10000 30000; do
    step rules $n
    timeout -k 10 300 python bench.py --config 2 --rules $n --no-cpu > "$O/bench_rules$n.json" 2> "$O/bench_rules$n.err" \
        || { tail -20 "$O/bench_rules$n.err"; exit 1; }
    grep -o '"value": [0-9.]*' "$O/bench_rules$n.json"; grep -o '"classifier": "[^}]*}' "$O/bench_rules$n.json"
done
step done
