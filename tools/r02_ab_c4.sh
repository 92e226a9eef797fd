# config 4 launch shape: workgroup size, root stride (LDS per workgroup), prefetch, lockstep chunk
set -o pipefail
O=gpurun_out/abc4; mkdir -p $O
run() { VPP_AMD_LIB=$PWD/vpp_amd/$1 timeout -k 10 200 python tools/sweep.py --config 4 --rounds 2 --reps 10 "${@:2}" | sed "s/^/$1 /" | tee -a $O/sweep.log; }
run libpolicygpu.so --tune block_stage=512,1024 || exit 1
run libpolicygpu.so --pre root_bits_max=12 --tune block_stage=512,1024 || exit 1
for lib in libpolicygpu_pf1.so libpolicygpu_q4.so libpolicygpu_q1.so libpolicygpu.so; do run $lib || exit 1; done
