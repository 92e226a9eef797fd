set -o pipefail
for L in libpolicygpu.so libpolicygpu_nogather.so libpolicygpu_nowalk.so libpolicygpu_nowalknogather.so libpolicygpu_probe0.so; do
  VPP_AMD_LIB=vpp_amd/$L timeout -k 10 200 python tools/sweep.py --config 3 --rounds 3 --reps 10 || exit 1
done
