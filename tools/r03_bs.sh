set -o pipefail
O=gpurun_out/r03_bs; mkdir -p $O
for spec in "2" "2 --rules 10000" "2 --rules 100000" "3" "6"; do
  echo "[$(date +%T)] config $spec"
  timeout -k 10 300 python tools/sweep.py --config $spec --tune block_stage=0,1024 --rounds 3 --reps 5 >> $O/sweep.jsonl 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
done
python -c "
import json
for l in open('$O/sweep.jsonl'):
    d=json.loads(l); print(d['config'], d.get('rules'), d['block_stage'], d['gpps'], d['out_sha'], d['same_output'])
"
