#!/bin/bash
# Compact FTRAN operand: its GPU tests, the whole GPU suite, then C3 bench
# lines with it on and off (SPX_DENSE_FTRAN=1), interleaved.
set -o pipefail
T=${1:-compact}
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$T"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_compact.py -x -v --timeout 200 --timeout-method thread > "$OUT/compact.log" 2>&1 || { tail -40 "$OUT/compact.log"; exit 1; }
tail -2 "$OUT/compact.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for r in 1 2; do
  for d in 0 1; do
    SPX_DENSE_FTRAN=$d timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-tableau --no-explicit --no-sharded-pricing > "$OUT/b_${d}_${r}.log" 2>&1 || { tail -20 "$OUT/b_${d}_${r}.log"; exit 1; }
    python3 -c "
import json;d=json.loads([l for l in open('$OUT/b_${d}_${r}.log') if l.startswith('{')][-1]);k=d['kernels']
print(json.dumps({'dense_ftran':$d,'it_s':round(d['value'],1),'price_us':round(d['roofline']['avg_launch_ms']*1e3,2),'update_us':round(k['k_update']['avg_launch_ms']*1e3,2),'fold_us':round(k['k_fold']['avg_launch_ms']*1e3,2)}))"
  done
done
