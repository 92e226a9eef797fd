set -o pipefail
O=gpurun_out/r03_pod; mkdir -p $O
for lib in libpolicygpu.so libpolicygpu_pf0w8.so; do
for spec in "3" "3 --counters" "6" "6 --counters"; do
  echo "[$(date +%T)] $lib config $spec"
  VPP_AMD_LIB=$(pwd)/vpp_amd/$lib timeout -k 10 300 python tools/sweep.py --config $spec --tune block_stage=0,1024 --rounds 3 --reps 5 >> $O/sweep.jsonl 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
done
done
python -c "
import json
for l in open('$O/sweep.jsonl'):
    d=json.loads(l); print(d['lib'], d['config'], d['counters'], d['block_stage'], d['gpps'], d['out_sha'])
"
