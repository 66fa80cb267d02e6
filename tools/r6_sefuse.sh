# Steepest edge: k_se_part's sums fused into k_ftran_bc (Params::se_fused,
# spx_api.cpp se_chain) against HEAD (xold): the steepest / group / mailbox /
# deferred-tail GPU tests, steepest and Dantzig passes (pass_ab), the bench's
# steepest block and C3 line alternating, SPX_SE_FUSE=0 as a third leg.
set -o pipefail
OUT=gpurun_out/${1:-r6sefuse}
mkdir -p $OUT
X=$PWD/simplex_method_gpu_amd/_ab/xold/libsimplex.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_steepest.py tests/test_gpu_pricing_groups.py tests/test_gpu_mbox.py tests/test_gpu_defer.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
PASS_AB_PRICING=2 timeout -k 10 500 python3 tools/pass_ab.py default $X env:SPX_SE_FUSE=0 || exit 1
timeout -k 10 500 python3 tools/pass_ab.py default $X || exit 1
for r in 1 2; do for L in default xold; do
  if [ $L = default ]; then LIB=""; else LIB=$X; fi
  SPX_LIB=$LIB timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-tableau --no-explicit --no-sharded-pricing > $OUT/b_${L}_$r.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['steepest']; t=d['solve_to_optimum']; print(sys.argv[2], 'C3', round(d['value']), round(d['roofline']['frac'],4), 'solve', round(t['seconds'],4), '| steepest', round(s['k_price_GBps']), round(s['value']), round(1e3*s['ms_per_step'],2), 'us, solve', s['solve']['pivots'], round(s['solve']['seconds'],4), s['solve']['z'])" $OUT/b_${L}_$r.json $L
done; done
