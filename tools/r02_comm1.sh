#!/bin/bash
# The multi-rank bench path (NCCL process group, RCCL all-gather MINLOC captured
# in hipGraphs, replicated window B^-1) with one rank, default build vs
# _build/<variant>.  usage: tools/r02_comm1.sh TAG variant
set -o pipefail
T=${1:-comm1}
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$T"
mkdir -p "$OUT"
cd "$ROOT"
for r in 1 2; do
  for v in default $2; do
    if [ $v = default ]; then L=$ROOT/simplex_method_gpu_amd/libsimplex.so; else L=$ROOT/simplex_method_gpu_amd/_build/$v/libsimplex.so; fi
    SPX_LIB=$L timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
        bench.py --comm1 --no-cpu-baseline --no-tableau --no-explicit > "$OUT/c_${v}_${r}.log" 2>&1 || { tail -20 "$OUT/c_${v}_${r}.log"; exit 1; }
    python3 -c "
import json;d=json.loads([l for l in open('$OUT/c_${v}_${r}.log') if l.startswith('{')][-1]);k=d['kernels'];pr=d['pricing']
print(json.dumps({'lib':'$v','it_s':round(d['value'],1),'dispatch':d['config']['dispatch'],'price_us':round(d['roofline']['avg_launch_ms']*1e3,2),'price_minloc_us':round(pr['max_rank_price_plus_minloc_ms']*1e3,2),'update_us':round(k['k_update']['avg_launch_ms']*1e3,2)}))"
  done
done
