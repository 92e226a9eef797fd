set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t9.log 2>&1 || { tail -30 gpurun_out/t9.log; exit 1; }
tail -2 gpurun_out/t9.log
for c in 2 6 3 5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($c, d['value'], d['roofline']['frac'], d['config']['classifier'][:80])" || exit 1
done
