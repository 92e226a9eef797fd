#!/bin/bash
# GPU tests, then the cold-start transient of the production kernel vs the stream-only probe
# build (same loads/stores, no classification), and the effective clock per dispatch of the
# driver's bench command (GRBM_GUI_ACTIVE / 8 / duration).
#   gpurun --timeout 900 -- bash tools/r02_diag2.sh TAG
set -o pipefail
TAG=${1:-diag2}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
step() { echo "[$(date +%T)] $*"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1 || { tail -30 "$O/gpu_tests.log"; exit 1; }
tail -2 "$O/gpu_tests.log"
for lib in libpolicygpu.so libpolicygpu_probe.so; do
    step ramp $lib
    VPP_AMD_LIB=$R/vpp_amd/$lib timeout -k 10 180 python tools/ramp_probe.py --config 2 > "$O/ramp_$lib.json" \
        2> "$O/ramp_$lib.err" || { tail -20 "$O/ramp_$lib.err"; exit 1; }
    python -c "
import json
for l in open('$O/ramp_$lib.json'):
    d=json.loads(l); print(d['phase'], d['summary_us'], d['us'][:30:3])
"
done
cd /tmp && export TMPDIR=/tmp
step pmc clock
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d "$O/clk_drv" -o run -- \
    python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu > "$O/clk_drv.log" 2>&1 \
    || { tail -20 "$O/clk_drv.log"; exit 1; }
step done
