#!/bin/bash
# Where the node kernels' time goes: measurement builds (no trie walks / no cross gathers /
# streams only) vs production, configs 3, 5 (with counters), 6; and the config-4 bench line.
set -o pipefail
TAG=${1:-probenode}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
step() { echo "[$(date +%T)] $*"; }
for lib in libpolicygpu.so libpolicygpu_pnowalk.so libpolicygpu_pnogather.so libpolicygpu_pboth.so libpolicygpu_pstream.so; do
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
step tests config 4
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q -k "config4" --timeout 300 \
    --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { tail -30 "$O/gpu_tests.log"; exit 1; }
tail -2 "$O/gpu_tests.log"
step bench config 4
timeout -k 10 300 python bench.py --config 4 --no-cpu > "$O/bench_c4.json" 2> "$O/bench_c4.err" || { tail -20 "$O/bench_c4.err"; exit 1; }
grep -o '"value": [0-9.]*' "$O/bench_c4.json"; grep -o '"roofline": {[^}]*}' "$O/bench_c4.json"
step done
