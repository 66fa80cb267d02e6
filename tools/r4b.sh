set -o pipefail
OUT=gpurun_out/r4b
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python3 -u tools/pass_ab.py env:SPX_DENSE_FOLD=1 env:SPX_DENSE_FOLD=0 > $OUT/ab_fold.log 2>&1 || { tail -30 $OUT/ab_fold.log; exit 1; }
cat $OUT/ab_fold.log
SPX_LIB=simplex_method_gpu_amd/_build/xmrg/libsimplex.so timeout -k 10 120 python3 -u tools/wg_probe.py > $OUT/wg_probe_mrg.json 2>&1 || { tail -30 $OUT/wg_probe_mrg.json; exit 1; }
head -20 $OUT/wg_probe_mrg.json
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels']['k_fold'], d['solve_to_optimum']['iterations_per_s'], d['solve_to_optimum']['seconds'])"
timeout -k 10 400 python3 -u bench.py --gpus 1 --config C5 --steps 63 --warmup 5 --no-explicit --no-tableau --no-cpu-baseline --no-steepest --no-sharded-pricing --no-solve-to-optimum > $OUT/bench_c5.log 2>&1 || { tail -30 $OUT/bench_c5.log; exit 1; }
grep '^{' $OUT/bench_c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels']['k_fold'])"
timeout -k 10 300 python3 -u tools/pass_ab.py default simplex_method_gpu_amd/_build/xtrim/libsimplex.so > $OUT/ab_trim.log 2>&1 || { tail -30 $OUT/ab_trim.log; exit 1; }
cat $OUT/ab_trim.log
timeout -k 10 300 python3 -u tools/pass_ab.py default simplex_method_gpu_amd/_build/xdeep/libsimplex.so > $OUT/ab_deep.log 2>&1 || { tail -30 $OUT/ab_deep.log; exit 1; }
cat $OUT/ab_deep.log
SPX_LIB=simplex_method_gpu_amd/_build/xdeep/libsimplex.so timeout -k 10 600 python -u -m pytest tests/test_gpu_defer.py tests/test_gpu_configs.py tests/test_gpu_compact.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_deep.log 2>&1 || { tail -40 $OUT/pytest_deep.log; exit 1; }
tail -2 $OUT/pytest_deep.log
SPX_LIB=simplex_method_gpu_amd/_build/xfsum/libsimplex.so timeout -k 10 120 python3 -u tools/wg_probe.py > $OUT/wg_probe_fsum.json 2>&1 || { tail -30 $OUT/wg_probe_fsum.json; exit 1; }
head -60 $OUT/wg_probe_fsum.json | grep -A3 ftran
timeout -k 10 400 python3 -u tools/ab.py --m 16384 --n 65536 --k 126 --warm 64 --rounds 3 --variants '[{}, {"_env": {"SPX_DENSE_FOLD": "1"}}, {"_env": {"SPX_FTRAN_RPW": "2"}}, {"_env": {"SPX_FTRAN_RPW": "4"}}]' > $OUT/ab_c5.log 2>&1 || { tail -30 $OUT/ab_c5.log; exit 1; }
tail -8 $OUT/ab_c5.log
timeout -k 10 60 ./tools/dpp_sum_check > $OUT/dpp_sum_check.log 2>&1 || { cat $OUT/dpp_sum_check.log; exit 1; }
cat $OUT/dpp_sum_check.log
timeout -k 10 300 python3 -u tools/pass_ab.py default simplex_method_gpu_amd/_build/xdpp/libsimplex.so > $OUT/ab_dpp.log 2>&1 || { tail -30 $OUT/ab_dpp.log; exit 1; }
cat $OUT/ab_dpp.log
timeout -k 10 300 python3 -u tools/pass_ab.py default simplex_method_gpu_amd/_build/xmerge1/libsimplex.so > $OUT/ab_merge1.log 2>&1 || { tail -30 $OUT/ab_merge1.log; exit 1; }
cat $OUT/ab_merge1.log
