# node kernels' occupancy: no stream prefetch (fewer VGPRs: PERPOD 68 -> 55, CONN+counters 82 -> 69),
# forced 8 waves per SIMD, 512 vs 1024-thread workgroups
set -o pipefail
O=gpurun_out/abocc; mkdir -p $O
run() { VPP_AMD_LIB=$PWD/vpp_amd/$1 PG_DEBUG_LAUNCH=1 timeout -k 10 250 python tools/sweep.py --rounds 2 --reps 8 "${@:2}" 2> $O/launch_$1_$3.err | sed "s/^/$1 /" | tee -a $O/sweep.log; sort $O/launch_$1_$3.err | uniq -c | grep "pg launch" | tail -3; }
for lib in libpolicygpu.so libpolicygpu_pf0.so libpolicygpu_pf0w8.so; do
  run $lib --config 3 --tune block_stage=512,1024 || exit 1
  run $lib --config 5 --counters --tune block_stage=512,1024 || exit 1
done
for lib in libpolicygpu.so libpolicygpu_pf0.so; do run $lib --config 6 --tune block_stage=512,1024 || exit 1; done
