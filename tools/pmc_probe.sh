#!/bin/bash
# PMC passes (one rocprofv3 --pmc run each, counters within the per-block slot limits) over a
# short bench run of one config: where a classify kernel's cycles go.
#   gpurun -- bash tools/pmc_probe.sh TAG CONFIG [bench args...]
# Writes gpurun_out/TAG/pmc_c<CONFIG>_<pass>/ and gpurun_out/TAG/counters.txt; summarise with
#   python tools/pmc_table.py gpurun_out/TAG
set -o pipefail
TAG=${1:-probe}; C=${2:-3}; shift 2
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
[ -s "$O/counters.txt" ] || timeout -k 5 60 rocprofv3 -L > "$O/counters.txt" 2>&1 || true
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS"
  "TA_TA_BUSY TA_BUFFER_READ_WAVEFRONTS TD_TD_BUSY TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ GRBM_GUI_ACTIVE GRBM_COUNT"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i + 1))
  ok=""
  for c in $p; do
    if grep -q -w "$c" "$O/counters.txt"; then ok="$ok $c"; else echo "skip unknown counter $c"; fi
  done
  [ -n "$ok" ] || continue
  echo "[$(date +%T)] pass $i:$ok"
  timeout -s KILL 90 rocprofv3 --pmc $ok --output-format csv -d "$O/pmc_c${C}_p$i" -o run -- \
      python3 "$R/bench.py" --config "$C" --no-cpu --no-check --steps 3 --warmup 1 "$@" > "$O/pmc_c${C}_p$i.log" 2>&1 \
      || { tail -5 "$O/pmc_c${C}_p$i.log"; exit 1; }
done
echo done
