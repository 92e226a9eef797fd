# FD tables read from HBM (STAGE 5): lockstep chunk 1 / 2 / 4, prefetch; config 4 at the new defaults
set -o pipefail
O=gpurun_out/abfd5; mkdir -p $O
run() { VPP_AMD_LIB=$PWD/vpp_amd/$1 timeout -k 10 250 python tools/sweep.py --rounds 2 --reps 10 "${@:2}" | sed "s/^/$1 /" | tee -a $O/sweep.log; }
run libpolicygpu.so --config 4 || exit 1
for lib in libpolicygpu.so libpolicygpu_fdq1.so libpolicygpu_fdq4.so libpolicygpu_fdpf.so; do
  run $lib --config 2 --rules 100000 || exit 1
  run $lib --config 7 || exit 1
done
