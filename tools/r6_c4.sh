# C4 line, new build against xold (HEAD before the ranged deep loads), twice
# each: the event-timed pricing fraction's spread; then the C4 / C5 rocprofv3
# kernel stats (tools/r6_prof45.sh).
set -o pipefail
OUT=gpurun_out/${1:-r6c4}
mkdir -p $OUT
XOLD=$PWD/simplex_method_gpu_amd/_ab/xold/libsimplex.so
for r in 1 2; do for L in default xold; do
  if [ $L = default ]; then LIB=""; else LIB=$XOLD; fi
  SPX_LIB=$LIB timeout -k 10 400 python3 -u bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-tableau --no-solve-to-optimum > $OUT/c4_${L}_$r.log 2>&1 || { tail -20 $OUT/c4_${L}_$r.log; exit 1; }
  grep '^{' $OUT/c4_${L}_$r.log > $OUT/c4_${L}_$r.json
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['value'],1), 'price ms', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],3))" $OUT/c4_${L}_$r.json $L
done; done
bash tools/r6_prof45.sh
