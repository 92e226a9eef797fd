set -o pipefail
O=gpurun_out/r03_t3; mkdir -p $O
for c in 512 1024 2048 4096 8192; do
  echo "[$(date +%T)] cells $c"
  timeout -k 10 200 python tools/sweep.py --config 6 --counters --pre node_hist_cells=$c --tune node_common_lds_max=0,81920,131072 --rounds 3 --reps 5 --warmup 20 >> $O/sweep.jsonl 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
done
cat $O/sweep.jsonl | cut -c1-250
