set -o pipefail
O=gpurun_out/r03_t1; mkdir -p $O
bash tools/gpu_tests.sh r03_t1 || exit 1
for c in 2 5 3; do
  echo "[$(date +%T)] bench $c"
  timeout -k 10 300 python bench.py --config $c > $O/b$c.json 2> $O/b$c.err || { tail -20 $O/b$c.err; exit 1; }
done
echo "[$(date +%T)] torchrun rehearsal"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --config 5 > $O/tr5.json 2> $O/tr5.err || { tail -20 $O/tr5.err; exit 1; }
echo done
