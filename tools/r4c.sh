set -o pipefail
OUT=gpurun_out/r4c
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
B=simplex_method_gpu_amd/_build
timeout -k 10 600 python3 -u tools/pass_ab.py default $B/xnodeep/libsimplex.so $B/xnodpp/libsimplex.so $B/xrb8/libsimplex.so $B/xrb4/libsimplex.so > $OUT/ab.log 2>&1 || { tail -30 $OUT/ab.log; exit 1; }
tail -1 $OUT/ab.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/tr_default -o run -- python3 $GRAFT_REPO_ROOT/tools/pmc_run.py --k 130 > $GRAFT_REPO_ROOT/$OUT/tr_default.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/tr_default.log; exit 1; }
SPX_LIB=$GRAFT_REPO_ROOT/$B/xrb8/libsimplex.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/tr_rb8 -o run -- python3 $GRAFT_REPO_ROOT/tools/pmc_run.py --k 130 > $GRAFT_REPO_ROOT/$OUT/tr_rb8.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/tr_rb8.log; exit 1; }
cd $GRAFT_REPO_ROOT
for d in tr_default tr_rb8; do f=$(find $OUT/$d -name "*kernel_stats.csv" | head -1); echo $d; cut -d, -f1-8 $f | head -12; done
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels']['k_fold']['avg_launch_ms'], d['solve_to_optimum']['iterations_per_s'])"
timeout -k 10 120 python3 -u tools/wg_probe.py > $OUT/wg_probe.json 2>&1 || { tail -30 $OUT/wg_probe.json; exit 1; }
grep -A1 "pass_total\|price_span\|ftran_publish_max\"" $OUT/wg_probe.json
