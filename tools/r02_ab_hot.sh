# A/B: constant-table shortcut + hot counter slots in registers (node kernels)
set -o pipefail
O=gpurun_out/abhot; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "cluster or node_kernel" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { VPP_AMD_LIB=$PWD/vpp_amd/$1 timeout -k 10 200 python tools/sweep.py --config $2 --rounds 2 --reps 10 "${@:3}" | sed "s/^/$1 c$2 $3 /" | tee -a $O/sweep.log; }
for r in 1 2; do
  for lib in libpolicygpu_base.so libpolicygpu.so libpolicygpu_nohot.so; do run $lib 5 --counters || exit 1; done
  for lib in libpolicygpu_base.so libpolicygpu.so; do run $lib 5 || exit 1; run $lib 3 || exit 1; done
done
