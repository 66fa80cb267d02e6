set -o pipefail
OUT=gpurun_out/r4deep
mkdir -p $OUT
B=simplex_method_gpu_amd/_build
timeout -k 10 600 python -u -m pytest tests/test_gpu_c45.py tests/test_gpu_defer.py tests/test_gpu_large.py tests/test_gpu_compact.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
PASS_AB_M=16384 PASS_AB_N=65536 timeout -k 10 400 python3 -u tools/pass_ab.py default $B/xnodeep/libsimplex.so > $OUT/ab_c5.log 2>&1 || { tail -30 $OUT/ab_c5.log; exit 1; }
tail -1 $OUT/ab_c5.log
timeout -k 10 300 python3 -u tools/pass_ab.py default $B/xnodeep/libsimplex.so > $OUT/ab_c3.log 2>&1 || { tail -30 $OUT/ab_c3.log; exit 1; }
tail -1 $OUT/ab_c3.log
