# wave-aggregated global counter atomics only for node kernels over oversized table sets
set -o pipefail
O=gpurun_out/abgagg2; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { VPP_AMD_LIB=$PWD/vpp_amd/$1 timeout -k 10 250 python tools/sweep.py --rounds 1 --reps 6 --warmup 10 "${@:2}" | sed "s/^/$1 /" | tee -a $O/sweep.log; }
for lib in libpolicygpu_base.so libpolicygpu.so; do
  run $lib --config 6 --counters || exit 1
  run $lib --config 4 --counters || exit 1
  run $lib --config 5 --counters || exit 1
done
