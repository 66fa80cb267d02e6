# SPX_PRICE_XCDMAP A/B, more rounds: four pass_ab sessions at C3 (12
# interleaved rounds) and three alternating bench C3 lines per build.
set -o pipefail
OUT=gpurun_out/${1:-r6xcd2}
mkdir -p $OUT
X=$PWD/simplex_method_gpu_amd/_ab/xxcd/libsimplex.so
for i in 1 2 3 4; do timeout -k 10 500 python3 tools/pass_ab.py default $X | tail -1 || exit 1; done
for r in 1 2 3; do for L in default xxcd; do
  if [ $L = default ]; then LIB=""; else LIB=$X; fi
  SPX_LIB=$LIB timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-tableau --no-explicit --no-sharded-pricing --no-steepest --no-solve-to-optimum > $OUT/b_${L}_$r.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'C3', round(d['value']), round(1e3*d['ms_per_step'],2), round(d['roofline']['frac'],4), [round(x) for x in d['timed_region']['next_windows_it_per_s']])" $OUT/b_${L}_$r.json $L
done; done
