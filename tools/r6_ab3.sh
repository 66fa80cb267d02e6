# Round-6 A/B session 3: WM 1 one-batch deep prefetch at the shard widths,
# k_ftran_bc U-row / chunk trims (PMC + pass time), steepest-edge deep batch.
set -o pipefail
OUT=gpurun_out/${1:-r6ab3}
mkdir -p $OUT
for L in default xdeep1; do
  if [ $L = default ]; then LIB=""; else LIB=$PWD/simplex_method_gpu_amd/_ab/$L/libsimplex.so; fi
  SPX_LIB=$LIB timeout -k 10 300 python3 tools/shard_rehearsal.py --n 16384 --gs 1,8 --price-grid 0,192 > $OUT/shard_$L.json 2>&1 || { tail -20 $OUT/shard_$L.json; exit 1; }
  python3 -c "import json; [print('$L', r['G'], r['price_grid'], r['shard_price_us']) for r in json.load(open('$OUT/shard_$L.json'))['rows']]"
done
bash tools/ftran_ab.sh ${1:-r6ab3}/ftran default xt2 xt3 || exit 1
bash tools/r6_se.sh ${1:-r6ab3}/se || exit 1
