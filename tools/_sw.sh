set -o pipefail
for c in 3 5; do for ns in 6 8; do
  timeout -k 10 200 python tools/sweep.py --config $c --ns $ns --tune node_local=1,0 --rounds 3 --reps 10 || exit 1
done; done
timeout -k 10 200 python tools/sweep.py --config 5 --ns 6 --counters --tune node_local=1,0 --rounds 3 --reps 10
