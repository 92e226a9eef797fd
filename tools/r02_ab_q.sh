# lockstep chunk after the LDS-addressing change: PERPOD 1 / 2 / 4, CONN (no counters) 1 / 2
set -o pipefail
O=gpurun_out/abq; mkdir -p $O
run() { VPP_AMD_LIB=$PWD/vpp_amd/$1 timeout -k 10 250 python tools/sweep.py --rounds 2 --reps 8 "${@:2}" | sed "s/^/$1 /" | tee -a $O/sweep.log; }
for lib in libpolicygpu.so libpolicygpu_qp1.so libpolicygpu_qp4.so; do run $lib --config 3 || exit 1; run $lib --config 6 || exit 1; done
for lib in libpolicygpu.so libpolicygpu_qc2.so; do run $lib --config 5 || exit 1; done
