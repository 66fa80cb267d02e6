# Fused mailbox exchange: the mailbox / comm / deferred-
# tail / group tests, then the multi-rank bench rehearsals on one GPU with the
# fused exchange and with the k_exchange launch (SPX_MBOX_FUSED=0), alternating:
# one rank (--comm1 --minloc mbox; RCCL beside it) and two ranks sharing GPU 0
# (those keep k_exchange: spx_mbox_attach sees the peer on the same device).
set -o pipefail
OUT=gpurun_out/${1:-r6mbox}
mkdir -p $OUT
export MASTER_ADDR=127.0.0.1
timeout -k 10 600 python -u -m pytest tests/test_gpu_mbox.py tests/test_gpu_comm.py tests/test_gpu_defer.py tests/test_gpu_pricing_groups.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
run1() {  # tag, env, extra bench args
  env $2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29511 bench.py --comm1 --steps 126 --warmup 5 --no-cpu-baseline --no-tableau --no-explicit --no-solve-to-optimum $3 \
      > $OUT/$1.log 2>&1 || { tail -30 $OUT/$1.log; return 1; }
  grep '^{' $OUT/$1.log | tail -1 > $OUT/$1.json
  python3 -c "import json; d=json.load(open('$OUT/$1.json')); g=d['config']['geometry']; print('$1', round(d['value'], 1), round(1e3 * d['ms_per_step'], 2), 'us/pivot; mbox_fused', g.get('mbox_fused'), 'next', [round(v) for v in d['timed_region']['next_windows_it_per_s']], 'price+minloc us', round(1e3*d['pricing']['max_rank_price_plus_minloc_ms'],2))"
}
for i in 1 2; do
  run1 comm1_mbox_fused "SPX_MBOX_FUSED=1" "--minloc mbox" || exit 1
  run1 comm1_mbox_kexch "SPX_MBOX_FUSED=0" "--minloc mbox" || exit 1
  run1 comm1_rccl "SPX_MBOX_FUSED=1" "" || exit 1
done
for f in 1; do
  SPX_MBOX_FUSED=$f timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 \
      bench.py --gpus 2 --share-gpu --steps 63 --warmup 5 --no-cpu-baseline --no-tableau --no-explicit > $OUT/share2_$f.log 2>&1 || { tail -30 $OUT/share2_$f.log; exit 1; }
  grep '^{' $OUT/share2_$f.log | tail -1 > $OUT/share2_$f.json
  python3 -c "import json; d=json.load(open('$OUT/share2_$f.json')); print('share2 fused=$f', round(d['value'], 1), d['n_gpus'], 'to_opt', d['solve_to_optimum']['pivots'], d['solve_to_optimum']['z'])"
done
