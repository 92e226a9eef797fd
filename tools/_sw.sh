set -o pipefail
mkdir -p gpurun_out/ab
run() { VPP_AMD_LIB=$PWD/vpp_amd/$1 timeout -k 10 200 python tools/sweep.py --config $2 --rounds 2 --reps 10 $3 | sed "s/^/$1 /" | tee -a gpurun_out/ab/sweep2.log; }
for r in 1 2; do
  for lib in libpolicygpu.so libpolicygpu_cq2ns.so; do run $lib 5 --counters || exit 1; done
  run libpolicygpu.so 5 "" || exit 1
  for c in 3 6; do for lib in libpolicygpu.so libpolicygpu_qp2.so; do run $lib $c "" || exit 1; done; done
done
