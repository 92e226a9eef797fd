set -o pipefail
for c in 2 4 3; do
for L in libpolicygpu_old.so libpolicygpu.so; do
  VPP_AMD_LIB=vpp_amd/$L timeout -k 10 200 python tools/sweep.py --config $c --rounds 5 --reps 10 || exit 1
done
done
