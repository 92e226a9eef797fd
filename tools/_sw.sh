set -o pipefail
for L in libpolicygpu.so libpolicygpu_s1.so libpolicygpu_s2.so; do
  VPP_AMD_LIB=vpp_amd/$L timeout -k 10 200 python tools/sweep.py --config 2 --tune block_stage=256,512,1024 --rounds 3 --reps 10 || exit 1
done
for L in libpolicygpu.so libpolicygpu_p1.so libpolicygpu_p2.so; do
  VPP_AMD_LIB=vpp_amd/$L timeout -k 10 200 python tools/sweep.py --config 3 --tune block_stage=256,512,1024 --rounds 3 --reps 5 || exit 1
done
VPP_AMD_LIB=vpp_amd/libpolicygpu.so timeout -k 10 200 python tools/sweep.py --config 5 --counters --tune block_stage=256,512,1024 --rounds 3 --reps 5 || exit 1
