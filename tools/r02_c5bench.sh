#!/bin/bash
# C5 bench lines (whole windows), default build vs _build/<variant>, interleaved.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/c5b
for r in 1 2; do for v in default $1; do
  if [ $v = default ]; then L=$ROOT/simplex_method_gpu_amd/libsimplex.so; else L=$ROOT/simplex_method_gpu_amd/_build/$v/libsimplex.so; fi
  SPX_LIB=$L timeout -k 10 300 python3 -u bench.py --config C5 --steps 126 --warmup 5 --no-cpu-baseline --no-tableau --no-explicit > gpurun_out/c5b/${v}_${r}.log 2>&1 || { tail -20 gpurun_out/c5b/${v}_${r}.log; exit 1; }
  python3 -c "
import json;d=json.loads([l for l in open('gpurun_out/c5b/${v}_${r}.log') if l.startswith('{')][-1]);k=d['kernels']
print(json.dumps({'lib':'$v','it_s':round(d['value'],1),'price_us':round(d['roofline']['avg_launch_ms']*1e3,1),'ftran_us':round(k['k_update']['avg_launch_ms']*1e3,1),'fold_us':round(k['k_fold']['avg_launch_ms']*1e3,1)}))"
done; done
