# CONN with counters at 32 waves per CU (64 registers, 1024-thread workgroups, no prefetch):
# lockstep chunk 2, and the same shape for CONN without counters
set -o pipefail
O=gpurun_out/abconn; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "cluster or node or conn" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { VPP_AMD_LIB=$PWD/vpp_amd/$1 timeout -k 10 250 python tools/sweep.py --rounds 2 --reps 8 "${@:2}" | sed "s/^/$1 /" | tee -a $O/sweep.log; }
for r in 1 2; do
for lib in libpolicygpu.so libpolicygpu_cq2.so libpolicygpu_cw6.so; do run $lib --config 5 --counters || exit 1; done
done
run libpolicygpu.so --config 5 || exit 1
run libpolicygpu_nc8.so --config 5 --tune block_stage=512,1024 || exit 1
run libpolicygpu.so --config 3 || exit 1
