# config 5 with counters: cost of the increments themselves (PG_PROBE_NOINC: every increment
# replaced by an untaken branch; the matched slot still computed; PG_PROBE_PLAINST: a plain LDS store in place of each atomic) vs the product, and without counters
set -o pipefail
O=gpurun_out/abnoinc2; mkdir -p $O
run() { VPP_AMD_LIB=$PWD/vpp_amd/$1 timeout -k 10 250 python tools/sweep.py --rounds 2 --reps 8 "${@:2}" | sed "s/^/$1 /" | tee -a $O/sweep.log; }
for r in 1 2; do for lib in libpolicygpu.so libpolicygpu_noinc.so libpolicygpu_plainst.so; do run $lib --config 5 --counters || exit 1; done; run libpolicygpu.so --config 5 || exit 1; done
