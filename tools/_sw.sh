set -o pipefail
for r in 1 2; do
for L in libpolicygpu.so libpolicygpu_pf1.so libpolicygpu_pf1s2.so libpolicygpu_probe0.so; do
  VPP_AMD_LIB=vpp_amd/$L timeout -k 10 200 python tools/sweep.py --config 2 --tune block_stage=512,1024 --rounds 5 --reps 20 || exit 1
done
done
