#!/bin/bash
# Profile pass per config: the bench line (driver settings), a rocprofv3 kernel trace with
# stats, FETCH_SIZE and WRITE_SIZE (separate passes, MI355X_MICROARCH.md HBM section), and
# utilisation passes (SQ: VALU / LDS / bank conflicts / wave cycles; TA / TD busy; GRBM
# cycles in each pass for the per-dispatch clock). Summarise with
#   python tools/prof_summary.py gpurun_out/TAG rNN_vK ; python tools/util_summary.py gpurun_out/TAG rNN_vK
#   gpurun --timeout 1200 -- bash tools/profile.sh TAG "2 4 3 5 6 2r10000 7" [extra bench args]
# A config spec NrM is config N at M rules (bench.py --config N --rules M: the rule-count sweep).
set -o pipefail
TAG=${1:-prof}; CONFIGS=${2:-2}; shift 2
EXTRA="$*"
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
step() { echo "[$(date +%T)] $*"; }
cd /tmp && export TMPDIR=/tmp
[ -s "$O/counters.txt" ] || timeout -k 5 60 rocprofv3 -L > "$O/counters.txt" 2>&1 || true
have() { grep -q -w "$1" "$O/counters.txt"; }
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU GRBM_GUI_ACTIVE"
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
  "TA_TA_BUSY TA_BUFFER_READ_WAVEFRONTS TD_TD_BUSY GRBM_GUI_ACTIVE GRBM_COUNT"
)
for c in $CONFIGS; do
    A="--config ${c%%r*}"; case $c in *r*) A="$A --rules ${c#*r}";; esac
    step bench config $c
    timeout -k 10 300 python3 "$R/bench.py" $A $EXTRA > "$O/bench_c$c.json" 2> "$O/bench_c$c.err" \
        || { tail -20 "$O/bench_c$c.err"; exit 1; }
    cut -c1-400 "$O/bench_c$c.json"
    step trace config $c
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c$c" -o run -- \
        python3 "$R/bench.py" $A --no-cpu --no-check $EXTRA > "$O/prof_c$c.log" 2>&1 \
        || { tail -20 "$O/prof_c$c.log"; exit 1; }
    for ctr in FETCH_SIZE WRITE_SIZE; do
        step pmc $ctr config $c
        timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$O/pmc_${ctr}_c$c" -o run -- \
            python3 "$R/bench.py" $A --no-cpu --no-check --steps 3 --warmup 1 $EXTRA > "$O/pmc_${ctr}_c$c.log" 2>&1 \
            || { tail -20 "$O/pmc_${ctr}_c$c.log"; exit 1; }
    done
    i=0
    for p in "${PASSES[@]}"; do
        i=$((i + 1))
        ok=""
        for k in $p; do if have "$k"; then ok="$ok $k"; else echo "skip unknown counter $k"; fi; done
        [ -n "$ok" ] || continue
        step util pass $i config $c
        timeout -s KILL 120 rocprofv3 --pmc $ok --output-format csv -d "$O/util_c${c}_p$i" -o run -- \
            python3 "$R/bench.py" $A --no-cpu --no-check --steps 3 --warmup 1 $EXTRA > "$O/util_c${c}_p$i.log" 2>&1 \
            || { tail -20 "$O/util_c${c}_p$i.log"; exit 1; }
    done
done
step done
