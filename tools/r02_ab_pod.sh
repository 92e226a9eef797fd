# PERPOD occupancy: one tuple per lockstep chunk (fewer registers), 64-register cap, prefetch
set -o pipefail
O=gpurun_out/abpod; mkdir -p $O
run() { VPP_AMD_LIB=$PWD/vpp_amd/$1 PG_DEBUG_LAUNCH=1 timeout -k 10 250 python tools/sweep.py --rounds 2 --reps 8 "${@:2}" 2> $O/l_$1_$3.err | sed "s/^/$1 /" | tee -a $O/sweep.log; sort $O/l_$1_$3.err | uniq -c | grep "pg launch" | tail -2; }
for lib in libpolicygpu.so libpolicygpu_pq1.so libpolicygpu_pq1w8.so libpolicygpu_pq1w8p0.so; do
  run $lib --config 3 --tune block_stage=512,1024 || exit 1
  run $lib --config 6 || exit 1
done
