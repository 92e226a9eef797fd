set -o pipefail
mkdir -p gpurun_out/ab
run() { timeout -k 10 200 python tools/sweep.py --config $1 --rounds 2 --reps 10 "${@:2}" | tee -a gpurun_out/ab/sweep3.log; }
for r in 1 2; do
  for m in 18 16 12; do run 4 --pre lc_max_stride=$m || exit 1; done
done
run 4 --pre lc_max_stride=16 --pre lc_dense12=64 || exit 1
run 4 --pre lc_max_stride=16 --pre root_bits_max=12 || exit 1
