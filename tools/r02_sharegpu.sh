#!/bin/bash
# bench.py's multi-rank path with 2 ranks sharing the one GPU of a pool box
# (--share-gpu: gloo process group, mailbox MINLOC), C3 and C2: the code the
# driver's --gpus N run executes, minus RCCL.  usage: tools/r02_sharegpu.sh [TAG]
set -o pipefail
T=${1:-share}
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$T"
mkdir -p "$OUT"
cd "$ROOT"
for c in C2 C3; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 \
      bench.py --gpus 2 --share-gpu --config $c --steps 126 --warmup 10 --no-cpu-baseline --no-tableau > "$OUT/$c.log" 2>&1 || { tail -30 "$OUT/$c.log"; exit 1; }
  grep '^{' "$OUT/$c.log" | tail -1 | python3 -c "
import json,sys;d=json.loads(sys.stdin.read())
print(json.dumps({'config':'$c','n_gpus':d['n_gpus'],'it_s':round(d['value'],1),'parallelism':d['config']['parallelism'],'dispatch':d['config']['dispatch'],'pricing':d['pricing'],'c4':d.get('pricing_c4'),'rehearsal':d.get('rehearsal')}))"
done
