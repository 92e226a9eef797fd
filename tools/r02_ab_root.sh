# config 4: LC root stride 12 / 13 / 14 (LDS per workgroup vs gathers per tuple)
set -o pipefail
O=gpurun_out/abroot; mkdir -p $O
run() { PG_DEBUG_LAUNCH=1 timeout -k 10 250 python tools/sweep.py --rounds 3 --reps 10 --config 4 "$@" 2> $O/l_$2.err | tee -a $O/sweep.log; sort $O/l_$2.err | uniq -c | grep "pg launch" | tail -1; }
for rb in 12 13 14; do run --pre lc_root_bits=$rb || exit 1; done
run --pre lc_root_bits=13 --tune block_stage=256,512,1024 || exit 1
