set -o pipefail
mkdir -p gpurun_out/geo
for c in 2 3 4 5 6; do
  PG_DEBUG_LAUNCH=1 timeout -k 10 200 python bench.py --config $c --no-cpu --steps 2 --warmup 1 > gpurun_out/geo/b$c.json 2> gpurun_out/geo/b$c.err || exit 1
  echo "config $c: $(grep 'pg launch' gpurun_out/geo/b$c.err | sort | uniq -c | tr '\n' ' ')"
done
