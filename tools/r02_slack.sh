#!/bin/bash
# Unit slack-column pricing: its GPU tests, then C3 bench lines with it on
# and off (SPX_DENSE_SLACKS=1), interleaved.  usage: tools/r02_slack.sh [TAG]
set -o pipefail
T=${1:-slack}
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$T"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_slack.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
for r in 1 2; do
  for d in 0 1; do
    SPX_DENSE_SLACKS=$d timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-tableau --no-explicit --no-sharded-pricing > "$OUT/b_${d}_${r}.log" 2>&1 || { tail -20 "$OUT/b_${d}_${r}.log"; exit 1; }
    python3 -c "
import json;d=json.loads([l for l in open('$OUT/b_${d}_${r}.log') if l.startswith('{')][-1]);k=d['kernels']
print(json.dumps({'dense_slacks':$d,'it_s':round(d['value'],1),'price_us':round(d['roofline']['avg_launch_ms']*1e3,2),'update_us':round(k['k_update']['avg_launch_ms']*1e3,2)}))"
  done
done
