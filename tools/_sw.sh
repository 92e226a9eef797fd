set -o pipefail
for L in libpolicygpu.so libpolicygpu_pf0.so libpolicygpu_tpl8.so libpolicygpu_tpl8pf0.so libpolicygpu_nopred.so libpolicygpu_nopredpf0.so libpolicygpu_probe0.so libpolicygpu_probe8.so; do
  VPP_AMD_LIB=vpp_amd/$L timeout -k 10 200 python tools/sweep.py --config 2 --tune block_stage=256,512,1024 --rounds 3 --reps 10 || exit 1
done
for L in libpolicygpu.so libpolicygpu_pf0.so libpolicygpu_tpl8.so libpolicygpu_tpl8pf0.so libpolicygpu_nopred.so; do
  for c in 3 5; do
    VPP_AMD_LIB=vpp_amd/$L timeout -k 10 200 python tools/sweep.py --config $c --tune block_stage=256,512,1024 --rounds 3 --reps 5 || exit 1
  done
done
