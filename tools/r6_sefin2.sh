# k_se_fin as 16 columns x 64 slices per workgroup (33 workgroups busy at C3
# instead of 9) against HEAD (xold): steepest pass (pass_ab) twice, the
# steepest-edge state after K pivots, the steepest / group tests.
set -o pipefail
OUT=gpurun_out/${1:-r6sefin2}
mkdir -p $OUT
X=$PWD/simplex_method_gpu_amd/_ab/xold/libsimplex.so
PASS_AB_PRICING=2 timeout -k 10 500 python3 tools/pass_ab.py default $X || exit 1
PASS_AB_PRICING=2 timeout -k 10 500 python3 tools/pass_ab.py default $X || exit 1
timeout -k 10 200 python3 tools/se_bits.py || exit 1
SPX_LIB=$X timeout -k 10 200 python3 tools/se_bits.py || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_steepest.py tests/test_gpu_pricing_groups.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
