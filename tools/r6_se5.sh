# k_price's deep prefetch as ranged buffer loads (0 bytes when the record is
# not fresh: the passes after the optimum) and the steepest-edge two-batch
# prefetch against the build before
# it (xold = HEAD): where the bench's steepest solve time goes (pivoting
# passes vs the passes after the optimum), pass times, the bench's steepest
# block, and the steepest / deferred-tail GPU tests.
set -o pipefail
OUT=gpurun_out/${1:-r6se5}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_steepest.py tests/test_gpu_defer.py tests/test_gpu_pricing_groups.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
XOLD=$PWD/simplex_method_gpu_amd/_ab/xold/libsimplex.so
for r in 1 2; do
  timeout -k 10 120 python3 tools/se_solve_split.py || exit 1
  SPX_LIB=$XOLD timeout -k 10 120 python3 tools/se_solve_split.py || exit 1
done
for r in 1 2; do
  timeout -k 10 120 python3 tools/se_solve_split.py 0 18291 || exit 1
  SPX_LIB=$XOLD timeout -k 10 120 python3 tools/se_solve_split.py 0 18291 || exit 1
done
timeout -k 10 500 python3 tools/pass_ab.py default $XOLD || exit 1
PASS_AB_PRICING=2 timeout -k 10 500 python3 tools/pass_ab.py default $XOLD || exit 1
for r in 1 2; do for L in default xold; do
  if [ $L = default ]; then LIB=""; else LIB=$XOLD; fi
  SPX_LIB=$LIB timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-tableau --no-explicit --no-sharded-pricing > $OUT/b_${L}_$r.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['steepest']; t=d['solve_to_optimum']; print(sys.argv[2], 'C3', round(d['value']), round(d['roofline']['frac'],4), 'solve', round(t['iterations_per_s']), round(t['seconds'],4), '| steepest', round(s['k_price_GBps']), round(s['value']), 'solve', round(s['solve']['seconds'],4))" $OUT/b_${L}_$r.json $L
done; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_all.log 2>&1 || { tail -30 $OUT/pytest_all.log; exit 1; }
tail -1 $OUT/pytest_all.log
