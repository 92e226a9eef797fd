#!/bin/bash
# PMC passes over A/B builds: for each library and config, one rocprofv3 --pmc run per pass
# (counters within the per-block slot limits), a short bench run each.
#   gpurun -- bash tools/pmc_libs.sh TAG "libA.so libB.so" "3 5c"
# PASSES (environment, ';'-separated counter lists) overrides the default passes.
# Writes gpurun_out/TAG/<lib>/pmc_c<C>_p<i>/; summarise with
#   for d in gpurun_out/TAG/*/; do python tools/pmc_table.py $d; done
set -o pipefail
TAG=${1:-pmclibs}; LIBS=${2:-libpolicygpu.so}; CONFIGS=${3:-3}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
[ -s "$O/counters.txt" ] || timeout -k 5 60 rocprofv3 -L > "$O/counters.txt" 2>&1 || true
DEF="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE;SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
IFS=';' read -r -a PS <<< "${PASSES:-$DEF}"
for lib in $LIBS; do
  for c in $CONFIGS; do
    cnt=""; case $c in *c) cnt="--counters";; esac
    i=0
    for p in "${PS[@]}"; do
      i=$((i + 1))
      ok=""
      for k in $p; do
        if grep -q -w "$k" "$O/counters.txt"; then ok="$ok $k"; else echo "skip unknown counter $k"; fi
      done
      [ -n "$ok" ] || continue
      mkdir -p "$O/${lib%.so}"
      echo "[$(date +%T)] $lib config $c pass $i:$ok"
      VPP_AMD_LIB=$R/vpp_amd/$lib timeout -s KILL 120 rocprofv3 --pmc $ok --output-format csv \
          -d "$O/${lib%.so}/pmc_c${c}_p$i" -o run -- \
          python3 "$R/bench.py" --config "${c%c}" $cnt --no-cpu --no-check --steps 3 --warmup 1 \
          > "$O/${lib%.so}/pmc_c${c}_p$i.log" 2>&1 || { tail -5 "$O/${lib%.so}/pmc_c${c}_p$i.log"; exit 1; }
    done
  done
done
echo done
