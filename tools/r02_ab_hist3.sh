# hit counters on the large tables: window + default-deny + last-rule cells
set -o pipefail
O=gpurun_out/abhist3; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { timeout -k 10 250 python tools/sweep.py --rounds 2 --reps 8 "$@" | tee -a $O/sweep.log; }
run --config 4 --counters || exit 1
run --config 2 --rules 100000 --counters || exit 1
run --config 2 --rules 100000 || exit 1
run --config 7 --counters || exit 1
run --config 7 || exit 1
