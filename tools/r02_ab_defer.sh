# CONN with counters: a connection's increments issued together after its last evalACL step
# (PG_CONN_DEFER=1) vs one after each step (default); config 3 with counters as a second case
set -o pipefail
O=gpurun_out/abdefer; mkdir -p $O
run() { VPP_AMD_LIB=$PWD/vpp_amd/$1 timeout -k 10 250 python tools/sweep.py --rounds 2 --reps 8 "${@:2}" | sed "s/^/$1 /" | tee -a $O/sweep.log; }
for r in 1 2; do for lib in libpolicygpu.so libpolicygpu_defer.so; do run $lib --config 5 --counters || exit 1; run $lib --config 3 --counters || exit 1; done; done
