#!/bin/bash
# Peer-mailbox MINLOC (spx_mbox_attach / k_exchange): its GPU tests, then the
# one-rank multi-rank bench path with the RCCL all-gather vs the mailbox
# exchange, interleaved.  usage: tools/r02_mbox.sh [TAG]
set -o pipefail
T=${1:-mbox}
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$T"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_mbox.py tests/test_gpu_comm.py -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
for r in 1 2; do
  for x in rccl mbox; do
    timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
        bench.py --comm1 --minloc $x --no-cpu-baseline --no-tableau --no-explicit > "$OUT/c_${x}_${r}.log" 2>&1 || { tail -20 "$OUT/c_${x}_${r}.log"; exit 1; }
    python3 -c "
import json;d=json.loads([l for l in open('$OUT/c_${x}_${r}.log') if l.startswith('{')][-1]);k=d['kernels'];pr=d['pricing']
print(json.dumps({'minloc':'$x','it_s':round(d['value'],1),'dispatch':d['config']['dispatch'],'price_us':round(d['roofline']['avg_launch_ms']*1e3,2),'price_minloc_us':round(pr['max_rank_price_plus_minloc_ms']*1e3,2),'update_us':round(k['k_update']['avg_launch_ms']*1e3,2),'c4':d.get('pricing_c4',{}).get('max_rank_price_plus_minloc_ms')}))"
  done
done
