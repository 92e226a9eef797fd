#!/bin/bash
# Node kernels A/B (out-of-line fallback vs inline; CONN chunks) + node GPU parity tests.
set -o pipefail
TAG=${1:-abnode2}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
step() { echo "[$(date +%T)] $*"; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kats.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { tail -30 "$O/gpu_tests.log"; exit 1; }
tail -2 "$O/gpu_tests.log"
for r in 1 2; do
for lib in libpolicygpu.so libpolicygpu_fbinl.so libpolicygpu_cc1.so libpolicygpu_qc2.so; do
    for c in 3 5c 5 6; do
        cnt=""; [ $c = 5c ] && cnt="--counters"
        step sweep $lib config $c
        VPP_AMD_LIB=$R/vpp_amd/$lib timeout -k 10 200 python tools/sweep.py --config ${c%c} --rounds 3 --reps 5 $cnt \
            >> "$O/sweep.jsonl" 2> "$O/sweep.err" || { tail -20 "$O/sweep.err"; exit 1; }
    done
done
done
python -c "
import json
for l in open('$O/sweep.jsonl'):
    d=json.loads(l); print(d['lib'], d['config'], d['counters'], d['ms'], d['gpps'])
"
step done
