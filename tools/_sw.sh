set -o pipefail
for c in 3 5; do for L in libpolicygpu.so libpolicygpu_gnt.so libpolicygpu.so libpolicygpu_gnt.so; do
  VPP_AMD_LIB=vpp_amd/$L timeout -k 10 200 python tools/sweep.py --config $c --rounds 3 --reps 10 || exit 1
done; done
