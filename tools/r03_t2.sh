set -o pipefail
O=gpurun_out/r03_t2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "large_node_set or cluster_configs or random_topology" > $O/t.log 2>&1; rc=$?; grep -E "PASSED|FAILED|Error|error" $O/t.log | tail -20; [ $rc -eq 0 ] || { tail -40 $O/t.log; exit 1; }
for args in "--config 6 --counters" "--config 6"; do
  echo "[$(date +%T)] bench $args"
  timeout -k 10 300 python bench.py $args --no-cpu > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  cut -c1-200 $O/b.json; grep -o '"parity_sample": {[^}]*}' $O/b.json
done
