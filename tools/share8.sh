# Rehearsal of the 8-GPU bench on a one-GPU box: 8 ranks share GPU 0
# (--share-gpu: gloo process group, mailbox MINLOC through IPC-mapped peer
# mailboxes; RCCL refuses two ranks on one device).  It runs the multi-rank
# bench path at world size 8 -- all_gather_object + check_ranks, the
# max-over-ranks clocks, solve_to_optimum and pricing_c4 at 8 ranks, rank-0
# output -- at C3 (default config: its pricing_c4 block shards C4 over the 8
# ranks) and at C4 (the config the verdict named; its own main line is the
# sharded C4 pricing, so pricing_c4 is not repeated, and the C4 solve to the
# optimum is left out: 8 ranks on one GPU take minutes for it).  Not a scaling
# number: the ranks share one GPU's bandwidth.   usage: tools/share8.sh [OUT]
set -o pipefail
OUT=${1:-gpurun_out/share8}
mkdir -p $OUT
export MASTER_ADDR=127.0.0.1 GPU_MAX_HW_QUEUES=1
run8() {  # tag, port, extra bench args
  timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
      --master-port $2 bench.py --gpus 8 --share-gpu --steps 20 --warmup 5 $3 > $OUT/$1.log 2>&1 \
      || { tail -40 $OUT/$1.log; return 1; }
  grep '^{' $OUT/$1.log | tail -1 > $OUT/$1.json
  python3 -c "import json; d=json.load(open('$OUT/$1.json')); r=d['ranks']; t=d.get('solve_to_optimum') or {}; p=d.get('pricing_c4') or {}; print('$1', 'world', r['world_size'], 'exchange', r['exchange'], 'ranks', [x['rank'] for x in r['per_rank']], 'value', round(d['value'], 1), 'to_opt', t.get('status'), t.get('pivots'), 'pricing_c4 GB/s', round(p.get('throughput_GBps', 0)))"
}
run8 share8_c3 29533 "" || exit 1
run8 share8_c4 29534 "--config C4 --no-solve-to-optimum" || exit 1
