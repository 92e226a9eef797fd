set -o pipefail
mkdir -p gpurun_out/ab
run() { VPP_AMD_LIB=$PWD/vpp_amd/$1 timeout -k 10 200 python tools/sweep.py --config $2 --rounds 2 --reps 10 "${@:3}" | sed "s/^/$1 /" | tee -a gpurun_out/ab/sweep4.log; }
for r in 1 2; do
  for c in 3 6; do for lib in libpolicygpu.so libpolicygpu_walk1.so; do run $lib $c || exit 1; done; done
  for lib in libpolicygpu.so libpolicygpu_walk1.so; do run $lib 5 --counters || exit 1; run $lib 5 || exit 1; done
done
