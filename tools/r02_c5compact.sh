#!/bin/bash
# C5 (and C4) with the compact FTRAN operand (default) against the dense
# stream's default (persistent k_loop at C5): bench lines, interleaved.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/c5c"
mkdir -p "$OUT"
cd "$ROOT"
for c in C5 C4; do
  for d in 0 1; do
    SPX_DENSE_FTRAN=$d timeout -k 10 300 python3 -u bench.py --config $c --steps 126 --warmup 5 --no-cpu-baseline --no-tableau --no-explicit --no-sharded-pricing > "$OUT/${c}_$d.log" 2>&1 || { tail -20 "$OUT/${c}_$d.log"; exit 1; }
    python3 -c "
import json;d=json.loads([l for l in open('$OUT/${c}_$d.log') if l.startswith('{')][-1]);k=d['kernels']
print(json.dumps({'config':'$c','dense_ftran':$d,'it_s':round(d['value'],1),'b_inverse':d['config']['b_inverse'][-80:],'dispatch':d['config']['dispatch'],'price_us':round(d['roofline']['avg_launch_ms']*1e3,1),'update_us':round(k['k_update']['avg_launch_ms']*1e3,1),'fold_us':round(k.get('k_fold',{}).get('avg_launch_ms',0)*1e3,1)}))"
  done
done
