# multi-rank bench rehearsals on a one-GPU box: the RCCL path with a one-rank communicator
# (--comm1; deferred and in-pass ratio-test tails, RCCL and mailbox MINLOC), and two ranks
# sharing GPU 0 (--share-gpu: gloo, mailbox MINLOC).  usage: tools/mr_rehearsal.sh
set -o pipefail
OUT=gpurun_out/mr
mkdir -p $OUT
export MASTER_ADDR=127.0.0.1
run1() {  # tag, env, extra bench args
  env $2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29511 bench.py --comm1 --steps 126 --warmup 5 --no-cpu-baseline --no-tableau --no-explicit $3 \
      > $OUT/$1.log 2>&1 || { tail -30 $OUT/$1.log; return 1; }
  grep '^{' $OUT/$1.log | tail -1 > $OUT/$1.json
  python3 -c "import json; d=json.load(open('$OUT/$1.json')); print('$1', round(d['value'], 1), round(1e3 * d['ms_per_step'], 2), 'us/pivot, defer_tail', d['config']['geometry']['defer_tail'])"
}
for i in 1 2; do
  run1 comm1_rccl_defer "SPX_DEFER_TAIL=1" "" || exit 1
  run1 comm1_rccl_inpass "SPX_DEFER_TAIL=0" "" || exit 1
  run1 comm1_mbox_defer "SPX_DEFER_TAIL=1" "--minloc mbox" || exit 1
done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 \
    bench.py --gpus 2 --share-gpu --steps 63 --warmup 5 --no-cpu-baseline --no-tableau > $OUT/share2.log 2>&1 || { tail -30 $OUT/share2.log; exit 1; }
grep '^{' $OUT/share2.log | tail -1 > $OUT/share2.json
python3 -c "import json; d=json.load(open('$OUT/share2.json')); print('share2', round(d['value'], 1), d['n_gpus'], d.get('rehearsal'))"
