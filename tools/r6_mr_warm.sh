# Multi-rank path first-span check: bench.py --comm1 (RCCL, one rank) with the
# default warm-up and with two more untimed windows before the timed span.
set -o pipefail
OUT=gpurun_out/${1:-r6mrw}
mkdir -p $OUT
export MASTER_ADDR=127.0.0.1
for i in 1 2; do for w in 5 131; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29511 bench.py --comm1 --steps 20 --warmup $w --no-cpu-baseline --no-tableau --no-explicit --no-solve-to-optimum --no-sharded-pricing \
      > $OUT/w$w_$i.log 2>&1 || { tail -30 $OUT/w$w_$i.log; exit 1; }
  grep '^{' $OUT/w$w_$i.log | tail -1 > $OUT/w${w}_$i.json
  python3 -c "import json; d=json.load(open('$OUT/w${w}_$i.json')); t=d['timed_region']; print('warmup $w', round(d['value'], 1), 'next', [round(v) for v in t['next_windows_it_per_s']], 'before', t['untimed_pivots_before'])"
done; done
