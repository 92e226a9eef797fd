# node image shape for configs 3 / 5: level-compressed IPv4 trie, root stride
set -o pipefail
O=gpurun_out/abnode3; mkdir -p $O
run() { timeout -k 10 250 python tools/sweep.py --rounds 2 --reps 8 "$@" | tee -a $O/sweep.log; }
for c in 3 6; do
  run --config $c || exit 1
  run --config $c --pre lc_node=1 || exit 1
  run --config $c --pre node_root_bits=14 || exit 1
  run --config $c --pre lc_node=1 --pre node_root_bits=8 || exit 1
done
run --config 5 --counters --pre lc_node=1 || exit 1
run --config 5 --counters || exit 1
