# launch shape re-check after the LDS-addressing change: workgroup size, resident workgroups per CU
set -o pipefail
O=gpurun_out/abc2shape; mkdir -p $O
run() { timeout -k 10 250 python tools/sweep.py --rounds 3 --reps 10 "$@" | tee -a $O/sweep.log; }
run --config 2 --tune block_stage=256,512,1024 || exit 1
run --config 2 --tune blocks_per_cu=0,2 || exit 1
run --config 3 --tune block_stage=256,512 || exit 1
