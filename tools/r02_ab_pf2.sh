# node kernels: next group's loads issued after the first cross-entry gather (PG_PREFETCH=2) vs at the top (default)
set -o pipefail
O=gpurun_out/abpf2; mkdir -p $O
run() { VPP_AMD_LIB=$PWD/vpp_amd/$1 timeout -k 10 250 python tools/sweep.py --rounds 2 --reps 8 "${@:2}" | sed "s/^/$1 /" | tee -a $O/sweep.log; }
for r in 1 2; do for lib in libpolicygpu.so libpolicygpu_pf2.so; do run $lib --config 3 || exit 1; run $lib --config 6 || exit 1; run $lib --config 5 || exit 1; done; done
