# The steepest-edge two-batch deep prefetch and the record-gated deep loads as
# the default, against the build before them (xold = HEAD~): C3 Dantzig and
# steepest pass time, the bench's steepest block and solve, the solve window
# by window, and the steepest / deferred-tail / large GPU tests.
set -o pipefail
OUT=gpurun_out/${1:-r6se4}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_steepest.py tests/test_gpu_defer.py tests/test_gpu_large.py tests/test_gpu_pricing_groups.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 500 python3 tools/pass_ab.py default simplex_method_gpu_amd/_ab/xold/libsimplex.so || exit 1
PASS_AB_PRICING=2 timeout -k 10 500 python3 tools/pass_ab.py default simplex_method_gpu_amd/_ab/xold/libsimplex.so || exit 1
for r in 1 2; do for L in default xold; do
  if [ $L = default ]; then LIB=""; else LIB=$PWD/simplex_method_gpu_amd/_ab/$L/libsimplex.so; fi
  SPX_LIB=$LIB timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-tableau --no-explicit --no-sharded-pricing > $OUT/b_${L}_$r.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['steepest']; t=d['solve_to_optimum']; print(sys.argv[2], 'C3', round(d['value']), round(d['roofline']['frac'],4), 'solve', round(t['iterations_per_s']), round(t['seconds'],4), '| steepest', round(s['k_price_GBps']), round(s['value']), 'solve', round(s['solve']['seconds'],4))" $OUT/b_${L}_$r.json $L
done; done
