# node kernels with counters: the node-output table's last rule counted in a register vs not
set -o pipefail
O=gpurun_out/abhotnode; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { VPP_AMD_LIB=$PWD/vpp_amd/$1 timeout -k 10 250 python tools/sweep.py --rounds 2 --reps 8 "${@:2}" | sed "s/^/$1 /" | tee -a $O/sweep.log; }
for r in 1 2; do for lib in libpolicygpu.so libpolicygpu_nohotnode.so; do
  run $lib --config 3 --counters || exit 1
  run $lib --config 5 --counters || exit 1
  run $lib --config 6 --counters || exit 1
done; done
