set -o pipefail
for r in 1 2; do for c in 3 5 6; do for lib in libpolicygpu_fbq4.so libpolicygpu.so; do
  VPP_AMD_LIB=$PWD/vpp_amd/$lib timeout -k 10 200 python tools/sweep.py --config $c --rounds 2 --reps 10 $( [ $c = 5 ] && echo --counters ) | sed "s/^/$lib /" || exit 1
done; done; done
