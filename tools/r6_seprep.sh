# k_se_part / k_se_fin with their loads issued before the pending test,
# against HEAD (xold): bits after K steepest pivots (three sizes), the
# steepest pass (pass_ab), the steepest / pricing-group GPU tests.
set -o pipefail
OUT=gpurun_out/${1:-r6seprep}
mkdir -p $OUT
X=$PWD/simplex_method_gpu_amd/_ab/xold/libsimplex.so
timeout -k 10 200 python3 tools/se_bits.py || exit 1
SPX_LIB=$X timeout -k 10 200 python3 tools/se_bits.py || exit 1
PASS_AB_PRICING=2 timeout -k 10 500 python3 tools/pass_ab.py default $X || exit 1
PASS_AB_PRICING=2 timeout -k 10 500 python3 tools/pass_ab.py default $X || exit 1
true

