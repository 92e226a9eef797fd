# config 2: resident 512-thread workgroups per CU (1 / 2 / 3 = occupancy), repeated
set -o pipefail
O=gpurun_out/abbpc; mkdir -p $O
for r in 1 2 3; do timeout -k 10 250 python tools/sweep.py --rounds 3 --reps 10 --config 2 --tune blocks_per_cu=3,2,1 | tee -a $O/sweep.log || exit 1; done
timeout -k 10 250 python tools/sweep.py --rounds 3 --reps 10 --config 2 --counters --tune blocks_per_cu=3,2 | tee -a $O/sweep.log || exit 1
