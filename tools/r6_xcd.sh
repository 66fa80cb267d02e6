# k_price's slot ranks by XCD (SPX_PRICE_XCDMAP=1, build xxcd) against the
# default: C3 pass (twice), the per-workgroup clock (XCD end means), C4 / C5
# passes, and the bench's C3 line alternating.
set -o pipefail
OUT=gpurun_out/${1:-r6xcd}
mkdir -p $OUT
X=$PWD/simplex_method_gpu_amd/_ab/xxcd/libsimplex.so
timeout -k 10 500 python3 tools/pass_ab.py default $X || exit 1
timeout -k 10 500 python3 tools/pass_ab.py default $X || exit 1
for L in default xxcd; do
  if [ $L = default ]; then LIB=""; else LIB=$X; fi
  SPX_LIB=$LIB timeout -k 10 120 python3 tools/wg_probe.py > $OUT/wg_$L.json 2>&1 || { tail -5 $OUT/wg_$L.json; exit 1; }
  python3 -c "
import json,sys
t=open(sys.argv[1]).read(); d=json.loads(t[t.index('{'):])
print(sys.argv[2], 'span', d['price_span']['p50'], 'end spread', d['price_end_spread']['p50'], 'pass', d['pass_total']['p50'], 'xcd', d['price_end_by_xcd'], 'p10/50/90/max', d['price_end_p10_p50_p90_max'])" $OUT/wg_$L.json $L
done
PASS_AB_N=131072 timeout -k 10 500 python3 tools/pass_ab.py default $X || exit 1
PASS_AB_M=16384 PASS_AB_N=65536 timeout -k 10 600 python3 tools/pass_ab.py default $X || exit 1
for r in 1 2; do for L in default xxcd; do
  if [ $L = default ]; then LIB=""; else LIB=$X; fi
  SPX_LIB=$LIB timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-tableau --no-explicit --no-sharded-pricing --no-steepest > $OUT/b_${L}_$r.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); t=d['solve_to_optimum']; print(sys.argv[2], 'C3', round(d['value']), round(1e3*d['ms_per_step'],2), round(d['roofline']['frac'],4), [round(x) for x in d['timed_region']['next_windows_it_per_s']], 'solve', round(t['seconds'],4))" $OUT/b_${L}_$r.json $L
done; done
