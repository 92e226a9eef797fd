#!/bin/bash
# VALU / LDS / memory-unit utilisation of the classify kernel: rocprofv3 derived metrics, one
# --pmc pass each (counters within the per-block slot limits), over a short bench run.
#   gpurun -- bash tools/util_probe.sh TAG "CONFIGS"
# Writes gpurun_out/TAG/util_c<C>_<metric>/ ; summarise with
#   python tools/util_summary.py gpurun_out/TAG PREFIX
set -o pipefail
TAG=${1:-util}; CONFIGS=${2:-2 3}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
[ -s "$O/counters.txt" ] || timeout -k 5 60 rocprofv3 -L > "$O/counters.txt" 2>&1 || true
PASSES=(VALUBusy VALUUtilization SALUBusy LDSBankConflict ALUStalledByLDS MemUnitBusy MemUnitStalled
        "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"
        "SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY")
for C in $CONFIGS; do
  i=0
  for p in "${PASSES[@]}"; do
    i=$((i + 1))
    ok=""
    for c in $p; do
      if grep -q -w "$c" "$O/counters.txt"; then ok="$ok $c"; else echo "skip unknown counter $c"; fi
    done
    [ -n "$ok" ] || continue
    echo "[$(date +%T)] config $C pass $i:$ok"
    timeout -s KILL 90 rocprofv3 --pmc $ok --output-format csv -d "$O/util_c${C}_p$i" -o run -- \
        python3 "$R/bench.py" --config "$C" --no-cpu --no-check --steps 3 --warmup 1 > "$O/util_c${C}_p$i.log" 2>&1 \
        || { tail -5 "$O/util_c${C}_p$i.log"; exit 1; }
  done
done
echo done
