# A/B: CANDI (inline candidates) vs the record form on config 4 and the large sweep tables;
# GPU parity of configs 2/4 (test_gpu_configs) first
set -o pipefail
O=gpurun_out/abcandi; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { timeout -k 10 200 python tools/sweep.py --config 4 --rounds 3 --reps 10 "$@" | tee -a $O/sweep.log; }
for r in 1 2; do run --pre candi=1 || exit 1; run --pre candi=0 || exit 1; done
timeout -k 10 300 python bench.py --config 4 > $O/bench_c4.json 2> $O/b4.err && cut -c1-600 $O/bench_c4.json
