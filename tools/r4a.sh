set -o pipefail
OUT=gpurun_out/r4a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
tail -c 3000 $OUT/bench.log
timeout -k 10 120 python3 -u tools/wg_probe.py > $OUT/wg_probe.json 2>&1 || { tail -30 $OUT/wg_probe.json; exit 1; }
head -40 $OUT/wg_probe.json
SPX_FTRAN_RPW=4 timeout -k 10 120 python3 -u tools/wg_probe.py > $OUT/wg_probe_rpw4.json 2>&1 || { tail -30 $OUT/wg_probe_rpw4.json; exit 1; }
head -30 $OUT/wg_probe_rpw4.json
timeout -k 10 300 python3 -u tools/pass_ab.py env:SPX_FTRAN_RPW=1 env:SPX_FTRAN_RPW=2 env:SPX_FTRAN_RPW=4 > $OUT/ab_rpw.log 2>&1 || { tail -30 $OUT/ab_rpw.log; exit 1; }
cat $OUT/ab_rpw.log
timeout -k 10 300 python3 -u tools/pass_ab.py default simplex_method_gpu_amd/_build/xsxe/libsimplex.so > $OUT/ab_sxe.log 2>&1 || { tail -30 $OUT/ab_sxe.log; exit 1; }
cat $OUT/ab_sxe.log
SPX_LIB=simplex_method_gpu_amd/_build/xfst/libsimplex.so timeout -k 10 120 python3 -u tools/wg_probe.py > $OUT/wg_probe_fst.json 2>&1 || { tail -30 $OUT/wg_probe_fst.json; exit 1; }
head -30 $OUT/wg_probe_fst.json
