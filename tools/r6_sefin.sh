# k_se_fin loading 32 partials per slice at a time (one round trip for the
# fused path's 512) against HEAD (xold): bits after K steepest pivots, the
# steepest pass (pass_ab) twice.
set -o pipefail
X=$PWD/simplex_method_gpu_amd/_ab/xold/libsimplex.so
timeout -k 10 200 python3 tools/se_bits.py || exit 1
SPX_LIB=$X timeout -k 10 200 python3 tools/se_bits.py || exit 1
PASS_AB_PRICING=2 timeout -k 10 500 python3 tools/pass_ab.py default $X || exit 1
PASS_AB_PRICING=2 timeout -k 10 500 python3 tools/pass_ab.py default $X || exit 1
