# CONN with counters: 32 waves/CU shape (64 registers, 1024 threads, no prefetch) vs 16 waves/CU, after the LDS-addressing change
set -o pipefail
O=gpurun_out/abcw; mkdir -p $O
run() { VPP_AMD_LIB=$PWD/vpp_amd/$1 timeout -k 10 250 python tools/sweep.py --rounds 2 --reps 8 "${@:2}" | sed "s/^/$1 /" | tee -a $O/sweep.log; }
for r in 1 2; do for lib in libpolicygpu.so libpolicygpu_cw1.so; do run $lib --config 5 --counters || exit 1; done; done
