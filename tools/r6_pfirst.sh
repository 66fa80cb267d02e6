# SPX_PRICE_PFIRST (k_price waits for the FTRAN partials before its deep
# prefetch) at the C3/8 shard width and at C3: the shard rehearsal (G = 1, 8)
# both ways, alternating; the per-workgroup clocks at n' = 5632 both ways; the
# C3 pass (pass_ab) both ways.
set -o pipefail
OUT=gpurun_out/${1:-r6pf}
mkdir -p $OUT
for r in 1 2; do for v in 0 1; do
  SPX_PRICE_PFIRST=$v timeout -k 10 120 python3 tools/shard_rehearsal.py --m 4096 --n 16384 --gs 8,4 > $OUT/sr_${v}_$r.json || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('pfirst', sys.argv[2], [(r['G'], r['shard_price_us']) for r in d['rows']])" $OUT/sr_${v}_$r.json $v
done; done
for v in 0 1; do
  SPX_PRICE_PFIRST=$v timeout -k 10 120 python3 tools/wg_probe.py --n 5632 > $OUT/wg_$v.json 2>&1 || { tail -5 $OUT/wg_$v.json; exit 1; }
  python3 -c "
import json,sys
t=open(sys.argv[1]).read(); d=json.loads(t[t.index('{'):])
print('pfirst', sys.argv[2], {k: v['p50'] for k, v in d.items() if isinstance(v, dict) and 'p50' in v and k.startswith('price')})" $OUT/wg_$v.json $v
done
timeout -k 10 500 python3 tools/pass_ab.py env:SPX_PRICE_PFIRST=0 env:SPX_PRICE_PFIRST=1 || exit 1
