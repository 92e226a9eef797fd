# config 4 / large tables after CANDI + 12-bit LC root + 512-thread workgroups: lockstep chunk,
# prefetch; LC root 12 vs 14 on the FD sweep tables and config 7
set -o pipefail
O=gpurun_out/abc4b; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { VPP_AMD_LIB=$PWD/vpp_amd/$1 timeout -k 10 250 python tools/sweep.py --rounds 2 --reps 10 "${@:2}" | sed "s/^/$1 /" | tee -a $O/sweep.log; }
for lib in libpolicygpu.so libpolicygpu_q4.so libpolicygpu_pf1.so; do run $lib --config 4 || exit 1; done
for rb in 12 14; do
  run libpolicygpu.so --config 2 --rules 30000 --pre lc_root_bits=$rb || exit 1
  run libpolicygpu.so --config 2 --rules 100000 --pre lc_root_bits=$rb || exit 1
  run libpolicygpu.so --config 7 --pre lc_root_bits=$rb || exit 1
done
