#!/bin/bash
# FD kernel (STAGE 4) first look: GPU tests, cold-start transient, driver bench, A/B of chunk /
# prefetch builds and workgroup sizes (tools/sweep.py, one process per build).
set -o pipefail
TAG=${1:-abfd}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
step() { echo "[$(date +%T)] $*"; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { tail -30 "$O/gpu_tests.log"; exit 1; }
tail -2 "$O/gpu_tests.log"
step bench driver command
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_drv.json" 2> "$O/bench_drv.err" \
    || { tail -20 "$O/bench_drv.err"; exit 1; }
cat "$O/bench_drv.json"
step ramp
timeout -k 10 180 python tools/ramp_probe.py --config 2 > "$O/ramp.json" 2> "$O/ramp.err" || { tail -20 "$O/ramp.err"; exit 1; }
python -c "
import json
for l in open('$O/ramp.json'):
    d=json.loads(l); print(d['phase'], d['summary_us'], d['us'][:30:3])
"
for r in 1 2; do
for lib in libpolicygpu.so libpolicygpu_qfd2.so libpolicygpu_qfd4.so libpolicygpu_pf1.so; do
    step sweep $lib
    VPP_AMD_LIB=$R/vpp_amd/$lib timeout -k 10 200 python tools/sweep.py --config 2 --rounds 3 --reps 10 \
        --tune block_stage=256,512,1024 >> "$O/sweep.jsonl" 2> "$O/sweep.err" || { tail -20 "$O/sweep.err"; exit 1; }
done
done
python -c "
import json
for l in open('$O/sweep.jsonl'):
    d=json.loads(l); print(d['lib'], d.get('block_stage'), d['ms'], d['gpps'], d['same_output'])
"
step done
