# resident workgroups per CU for configs 3 / 4 / 6 (occupancy = 3)
set -o pipefail
O=gpurun_out/abbpc2; mkdir -p $O
for c in 3 4 6; do timeout -k 10 250 python tools/sweep.py --rounds 3 --reps 8 --config $c --tune blocks_per_cu=0,2 | tee -a $O/sweep.log || exit 1; done
timeout -k 10 250 python tools/sweep.py --rounds 3 --reps 8 --config 5 --tune blocks_per_cu=0,3 | tee -a $O/sweep.log || exit 1
