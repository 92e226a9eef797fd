#!/bin/bash
# Driver-settings bench lines for several configs (and extra args), one after another:
#   gpurun -- bash tools/bench_set.sh TAG "2 3 5 6" [extra bench args]
# A config spec NrM is config N at M rules; a trailing c adds --counters.
set -o pipefail
TAG=${1:-bench}; CONFIGS=${2:-2}; shift 2
O=$(pwd)/gpurun_out/$TAG
mkdir -p "$O"
for c in $CONFIGS; do
    cc=${c%c}; A=""; case $c in *c) A="--counters";; esac
    A="$A --config ${cc%%r*}"; case $cc in *r*) A="$A --rules ${cc#*r}";; esac
    echo "[$(date +%T)] bench $A $*"
    timeout -k 10 300 python bench.py $A "$@" > "$O/b$c.json" 2> "$O/b$c.err" || { tail -20 "$O/b$c.err"; exit 1; }
    python - "$O/b$c.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(d["config"]["workload"][:40], "counters" if d["config"]["counters"] else "", d["value"], "frac", r["frac"],
      "of-probe", r.get("frac_of_measured_stream"), "parity", d.get("parity_sample", {}).get("bit_exact_action_and_rule_index"),
      d.get("parity_sample", {}).get("counters_equal_oracle_histogram"))
PY
done
