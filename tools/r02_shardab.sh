#!/bin/bash
# GPU tests, then the C3 shard rehearsal (tools/shard_rehearsal.py) and the C3
# rate for the default build and _build/<variant>.  usage: tools/r02_shardab.sh variant
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/shardab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/shardab/pytest.log 2>&1 || { tail -30 gpurun_out/shardab/pytest.log; exit 1; }
tail -1 gpurun_out/shardab/pytest.log
for v in default $1 $2; do
  if [ $v = default ]; then L=$ROOT/simplex_method_gpu_amd/libsimplex.so; else L=$ROOT/simplex_method_gpu_amd/_build/$v/libsimplex.so; fi
  SPX_LIB=$L timeout -k 10 300 python3 -u tools/shard_rehearsal.py --n 16384 > gpurun_out/shardab/$v.json || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/shardab/$v.json'));print('$v', [(r['G'], r['shard_price_us'], r['pricing_speedup_vs_1']) for r in d['rows']])"
  SPX_LIB=$L timeout -k 10 120 python3 tools/itbench.py --tag $v --reps 2 | grep '^{' || exit 1
done
