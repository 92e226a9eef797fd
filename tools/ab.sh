#!/bin/bash
# A/B of builds (tools/sweep.py in alternating processes) on the given configs, 2 rounds.
# Builds: make -C vpp_amd/csrc variant V=name DEFS="-DPG_...=..." -> vpp_amd/libpolicygpu_name.so
# Configs: 3, 5c (with counters), r10000 (config 2 at 10k rules), 9m2c (config 9 in mode 2, counted), ...
#   gpurun -- bash tools/ab.sh TAG "libA libB" "3 5c 6" [pytest paths]
# PRE="key=v ..." (environment): compiler knobs set before the tables are built (sweep.py --pre)
# TUNE="key=v1,v2 ..." (environment): launch knobs swept inside each run (sweep.py --tune)
# SWEEP="..." (environment): the sweep's own arguments (default --rounds 3 --reps 5 after 60
#   warm-up launches); SWEEP="--warmup 5 --rounds 1 --reps 20" times the driver's window
set -o pipefail
TAG=${1:-ablib}; LIBS=${2:-libpolicygpu.so}; CONFIGS=${3:-3}; TESTS=${4:-}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
step() { echo "[$(date +%T)] $*"; }
if [ -n "$TESTS" ]; then
    step tests $TESTS
    timeout -k 10 800 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread \
        > "$O/gpu_tests.log" 2>&1 || { tail -30 "$O/gpu_tests.log"; exit 1; }
    tail -2 "$O/gpu_tests.log"
fi
for r in $(seq ${ROUNDS:-2}); do
for lib in $LIBS; do
    for c in $CONFIGS; do
        cnt=""; case $c in *c) cnt="--counters";; esac
        extra=""; case $c in r*) extra="--rules ${c#r}"; c=2;; esac
        case $c in *m*) b=${c%c}; extra="$extra --mode ${b#*m}"; c=${b%m*};; esac
        step sweep $lib config $c $cnt $extra
        pre=""; for kv in ${PRE:-}; do pre="$pre --pre $kv"; done
        for kv in ${TUNE:-}; do pre="$pre --tune $kv"; done
        VPP_AMD_LIB=$R/vpp_amd/$lib timeout -k 10 200 python tools/sweep.py --config ${c%c} ${SWEEP:---rounds 3 --reps 5} $cnt $pre $extra \
            >> "$O/sweep.jsonl" 2> "$O/sweep.err" || { tail -20 "$O/sweep.err"; exit 1; }
    done
done
done
python -c "
import json
for l in open('$O/sweep.jsonl'):
    d = json.loads(l)
    t={k: v for k, v in d.items() if k not in ('lib', 'config', 'rules', 'counters', 'pre', 'ns', 'ms', 'gpps', 'GBps',
                                           'same_output', 'out_sha', 'blob')}
    print(d['lib'], d['config'], d.get('rules') or '', d['counters'], d['pre'], t or '', d['ms'], d['gpps'], d.get('out_sha'))
"
step done
