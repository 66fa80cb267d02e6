# Round-6 A/B session 1: k_ftran_bc trims (PMC + pass time), per-workgroup
# clocks at C3 (workgroup 0's deferred bookkeeping) and at the C3 / 8 shard
# width, and the shard rehearsal.
set -o pipefail
OUT=gpurun_out/${1:-r6ab1}
mkdir -p $OUT
timeout -k 10 200 python3 tools/wg_probe.py > $OUT/wg_c3.json 2>&1 || { tail -20 $OUT/wg_c3.json; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/wg_c3.json')); print('C3', {k: v['p50'] for k, v in d.items() if isinstance(v, dict) and 'p50' in v}); print('xcd', d['price_end_by_xcd'])"
timeout -k 10 200 python3 tools/wg_probe.py --n 5632 > $OUT/wg_c3s8.json 2>&1 || { tail -20 $OUT/wg_c3s8.json; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/wg_c3s8.json')); print('C3/8', {k: v['p50'] for k, v in d.items() if isinstance(v, dict) and 'p50' in v})"
timeout -k 10 300 python3 tools/shard_rehearsal.py --n 16384 --price-grid 0,96,192 > $OUT/shard_c3.json 2>&1 || { tail -20 $OUT/shard_c3.json; exit 1; }
cat $OUT/shard_c3.json
bash tools/ftran_ab.sh ${1:-r6ab1}/ftran default xt1 xt2 xt3
