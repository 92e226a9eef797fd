# hit counters: last-rule slot counted in a register (default) vs none (nohot) vs one round of
# wave aggregation (agg1, built before the register count)
set -o pipefail
O=gpurun_out/abagg; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "counters or sweep" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { VPP_AMD_LIB=$PWD/vpp_amd/$1 timeout -k 10 250 python tools/sweep.py --rounds 2 --reps 8 "${@:2}" | sed "s/^/$1 /" | tee -a $O/sweep.log; }
for r in 1 2; do for lib in libpolicygpu.so libpolicygpu_nohot.so libpolicygpu_agg1.so; do
  run $lib --config 2 --counters || exit 1
  run $lib --config 4 --counters || exit 1
done; done
run libpolicygpu.so --config 5 --counters || exit 1
run libpolicygpu_nohot.so --config 5 --counters || exit 1
