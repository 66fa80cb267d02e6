#!/bin/bash
# GPU tests, then interleaved bench lines (no CPU baseline / tableau / explicit
# blocks) of the default build and _build/<variant>: it/s and per-kernel times.
# usage: tools/r02_abbench.sh TAG variant [config]
set -o pipefail
T=${1:-abb}
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$T"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for r in 1 2; do
  for v in default $2 $3; do
    if [ $v = default ]; then L=$ROOT/simplex_method_gpu_amd/libsimplex.so; else L=$ROOT/simplex_method_gpu_amd/_build/$v/libsimplex.so; fi
    SPX_LIB=$L timeout -k 10 300 python3 -u bench.py --config C3 --no-cpu-baseline --no-tableau --no-explicit > "$OUT/b_${v}_${r}.log" 2>&1 || { tail -20 "$OUT/b_${v}_${r}.log"; exit 1; }
    python3 -c "
import json,sys;d=json.loads([l for l in open('$OUT/b_${v}_${r}.log') if l.startswith('{')][-1]);k=d['kernels']
print(json.dumps({'lib':'$v','it_s':round(d['value'],1),'price_us':round(d['roofline']['avg_launch_ms']*1e3,2),'update_us':round(k['k_update']['avg_launch_ms']*1e3,2),'fold_us':round(k['k_fold']['avg_launch_ms']*1e3,2) if k['k_fold'] else None}))"
  done
done
