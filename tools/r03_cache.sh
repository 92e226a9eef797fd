set -o pipefail
O=gpurun_out/r03_cache; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "large_node_set or cluster_configs or random_topolog" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
echo "[$(date +%T)] sweep"
timeout -k 10 300 python tools/sweep.py --config 6 --counters --tune node_hist_cells=0,256,512,1024,2048,4096,8192 --tune node_common_lds_max=0,81920 --rounds 3 --reps 5 > $O/sweep.jsonl 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
python -c "
import json
for l in open('$O/sweep.jsonl'):
    d=json.loads(l); print(d['node_hist_cells'], d['node_common_lds_max'], d['gpps'], d['out_sha'], d['same_output'])
"
