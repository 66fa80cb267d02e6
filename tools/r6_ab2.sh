# Round-6 A/B session 2: k_ftran_bc trims (fixed chunk fallback), narrow-shard
# geometries (price grid, no deep prefetch), the bench with its 252-pivot span.
set -o pipefail
OUT=gpurun_out/${1:-r6ab2}
mkdir -p $OUT
timeout -k 10 300 python3 tools/shard_rehearsal.py --n 16384 --gs 8 --price-grid 128,160,192,224,256 > $OUT/shard_g8.json 2>&1 || { tail -20 $OUT/shard_g8.json; exit 1; }
python3 -c "import json; [print(r) for r in json.load(open('$OUT/shard_g8.json'))['rows']]"
SPX_LIB=$PWD/simplex_method_gpu_amd/_ab/xnodeep/libsimplex.so timeout -k 10 300 python3 tools/shard_rehearsal.py --n 16384 --gs 1,8 --price-grid 0,192 > $OUT/shard_nodeep.json 2>&1 || { tail -20 $OUT/shard_nodeep.json; exit 1; }
python3 -c "import json; [print('nodeep', r) for r in json.load(open('$OUT/shard_nodeep.json'))['rows']]"
bash tools/ftran_ab.sh ${1:-r6ab2}/ftran default xt1 xt2 xt3 || exit 1
for c in C3 C3 C2; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-tableau --no-steepest --no-explicit --no-sharded-pricing > $OUT/bench_$c.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); t=d['timed_region']; print(sys.argv[2], round(d['value']), d['steps'], [round(v) for v in t['next_windows_it_per_s']], round(d['roofline']['frac'],3))" $OUT/bench_$c.json $c
done
