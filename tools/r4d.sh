set -o pipefail
OUT=gpurun_out/r4d
mkdir -p $OUT
timeout -k 10 120 python3 -u tools/cfold_probe.py > $OUT/cfold_c3.json 2>&1 || { tail -30 $OUT/cfold_c3.json; exit 1; }
cat $OUT/cfold_c3.json
SPX_LIB=simplex_method_gpu_amd/_build/xrb8/libsimplex.so timeout -k 10 120 python3 -u tools/cfold_probe.py > $OUT/cfold_c3_rb8.json 2>&1 || { tail -30 $OUT/cfold_c3_rb8.json; exit 1; }
cat $OUT/cfold_c3_rb8.json
timeout -k 10 200 python3 -u tools/cfold_probe.py --m 16384 --n 65536 > $OUT/cfold_c5.json 2>&1 || { tail -30 $OUT/cfold_c5.json; exit 1; }
cat $OUT/cfold_c5.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_window.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
