#!/bin/bash
# A/B of builds x tuning values (sweep.py --tune) on one config, 2 rounds.
#   gpurun -- bash tools/r02_ab_tune.sh TAG "libA libB" CONFIG "key=v1,v2" [--counters]
set -o pipefail
TAG=${1:-abtune}; LIBS=${2:-libpolicygpu.so}; CFG=${3:-5}; TUNE=${4:-block_stage=0}; CNT=${5:-}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
for r in 1 2; do
for lib in $LIBS; do
    echo "[$(date +%T)] sweep $lib config $CFG $TUNE $CNT"
    VPP_AMD_LIB=$R/vpp_amd/$lib timeout -k 10 300 python tools/sweep.py --config $CFG --rounds 3 --reps 5 \
        --tune "$TUNE" $CNT >> "$O/sweep.jsonl" 2> "$O/sweep.err" || { tail -20 "$O/sweep.err"; exit 1; }
done
done
python -c "
import json
for l in open('$O/sweep.jsonl'):
    d=json.loads(l); [d.pop(k, None) for k in ('pre', 'ns', 'GBps', 'blob')]; print(d)
"
echo "[$(date +%T)] done"
