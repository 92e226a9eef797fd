# config 2: FD shapes under smaller LDS budgets (more workgroups per CU, one or two more LDS
# reads per field); bench stdout under torchrun carries only the JSON line
set -o pipefail
O=gpurun_out/abfdshape; mkdir -p $O
run() { PG_DEBUG_LAUNCH=1 timeout -k 10 250 python tools/sweep.py --rounds 3 --reps 10 --config 2 "$@" 2> $O/l_$2.err | tee -a $O/sweep.log; sort $O/l_$2.err | uniq -c | grep "pg launch" | tail -2; }
for r in 1 2; do for smw in 16384 10240 8192; do run --pre stage_max_words=$smw || exit 1; done; done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 1 --no-cpu > $O/tr.json 2> $O/tr.err && wc -l $O/tr.json && cut -c1-120 $O/tr.json
