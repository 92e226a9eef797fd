# hit counters over more slots than the LDS histogram holds (config 4: 100k rules): LDS window
# of the table's first rules + default-deny cell, global atomics beyond; window size sweep
set -o pipefail
O=gpurun_out/abhist; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { PG_DEBUG_LAUNCH=1 timeout -k 10 250 python tools/sweep.py --rounds 2 --reps 8 "$@" 2> $O/l.err | tee -a $O/sweep.log; sort $O/l.err | uniq -c | grep "pg launch" | tail -1; }
for hw in 1024 4096 16383; do run --config 4 --counters --pre hist_window=$hw || exit 1; done
run --config 4 || exit 1
run --config 2 --counters || exit 1
run --config 5 --counters || exit 1
