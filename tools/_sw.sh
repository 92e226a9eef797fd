set -o pipefail
for r in 1 2; do
  VPP_AMD_LIB=vpp_amd/libpolicygpu_old.so timeout -k 10 200 python tools/sweep.py --config 4 --rounds 3 --reps 10 || exit 1
  VPP_AMD_LIB=vpp_amd/libpolicygpu.so timeout -k 10 200 python tools/sweep.py --config 4 --tune stage_root_max_words=16400,0 --rounds 3 --reps 10 || exit 1
done
