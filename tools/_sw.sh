set -o pipefail
for r in 1 2; do for d in 256 16; do
  timeout -k 10 200 python tools/sweep.py --config 4 --pre lc_dense12=$d --rounds 3 --reps 10 || exit 1
done; done
