# config 4: 64-register cap (four 512-thread workgroups per CU) vs none
set -o pipefail
O=gpurun_out/absw; mkdir -p $O
run() { VPP_AMD_LIB=$PWD/vpp_amd/$1 PG_DEBUG_LAUNCH=1 timeout -k 10 250 python tools/sweep.py --rounds 3 --reps 10 --config 4 "${@:2}" 2> $O/l_$1$2.err | sed "s/^/$1 /" | tee -a $O/sweep.log; sort $O/l_$1$2.err | uniq -c | grep "pg launch" | tail -1; }
for lib in libpolicygpu.so libpolicygpu_sw1.so; do run $lib || exit 1; run $lib --counters || exit 1; done
