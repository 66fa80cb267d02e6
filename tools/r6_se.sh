# Steepest-edge k_price A/B: the one-batch deep prefetch
# (SPX_PRICE_DEEP_SE=1, build xdse) against the default, pass time interleaved
# and the bench's steepest block (k_price GB/s, the whole solve), alternating.
set -o pipefail
OUT=gpurun_out/${1:-r6se}
mkdir -p $OUT
PASS_AB_PRICING=2 timeout -k 10 400 python3 tools/pass_ab.py default simplex_method_gpu_amd/_ab/xdse/libsimplex.so || exit 1
for r in 1 2 3; do for L in default xdse; do
  if [ $L = default ]; then LIB=""; else LIB=$PWD/simplex_method_gpu_amd/_ab/$L/libsimplex.so; fi
  SPX_LIB=$LIB timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-tableau --no-explicit --no-sharded-pricing --no-solve-to-optimum > $OUT/b_${L}_$r.json 2>/dev/null || exit 1
  python3 -c "import json,sys; s=json.load(open(sys.argv[1]))['steepest']; print(sys.argv[2], round(s['k_price_GBps']), round(1e3*s['k_price_ms'],2), 'us', round(s['value']), 'it/s solve', s['solve']['pivots'], round(s['solve']['seconds'],4))" $OUT/b_${L}_$r.json $L
done; done
