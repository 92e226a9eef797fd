#!/bin/bash
# Round-2 diagnosis of the slow first launches: per-launch durations (HIP events) in cold /
# idle / busy / regenerated phases, and a kernel trace of exactly the driver's bench command.
#   gpurun --timeout 600 -- bash tools/r02_diag.sh TAG
set -o pipefail
TAG=${1:-diag}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
step() { echo "[$(date +%T)] $*"; }
step ramp
timeout -k 10 180 python tools/ramp_probe.py --config 2 > "$O/ramp_c2.json" 2> "$O/ramp_c2.err" \
    || { tail -20 "$O/ramp_c2.err"; exit 1; }
python -c "
import json,sys
for l in open('$O/ramp_c2.json'):
    d=json.loads(l); print(d['phase'], d['summary_us'], d['us'][:12])
"
step bench driver command
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_drv.json" 2> "$O/bench_drv.err" \
    || { tail -20 "$O/bench_drv.err"; exit 1; }
cat "$O/bench_drv.json"
cd /tmp && export TMPDIR=/tmp
step trace driver command
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/trace_drv" -o run -- \
    python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu > "$O/trace_drv.log" 2>&1 \
    || { tail -20 "$O/trace_drv.log"; exit 1; }
step done
