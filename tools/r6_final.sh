# Round-6 final evidence on the final build (profiles of
# HEAD): rocprofv3 kernel stats and the PMC FETCH / WRITE passes first (so the
# bench lines read this build's traffic), then every -m gpu test (the full-size
# C4 / C5 certificates last), smoke(), the bench with the driver's arguments
# three times, and the C2 / C4 / C5 lines.
#   tools/r6_final.sh [OUT]   (OUT under gpurun_out/)
set -o pipefail
R=r06
OUT=gpurun_out/${1:-r6final}
mkdir -p $OUT
bash tools/gpu_profile.sh $R || exit 1
P=gpurun_out/prof_$R
TJ=$P/traffic_$R.json
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
for i in 1 2 3; do
  timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --traffic-json $TJ > $OUT/bench_$i.log 2>&1 || { tail -30 $OUT/bench_$i.log; exit 1; }
  grep '^{' $OUT/bench_$i.log > $OUT/bench_$i.json
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); t=d['timed_region']; print('C3', round(d['value']), round(1e3*d['ms_per_step'], 2), 'us', round(d['roofline']['frac'], 3), 'builds', t['graph_builds'], 'next', [round(v) for v in t['next_windows_it_per_s'] or []], 'to_opt', round(d['solve_to_optimum']['iterations_per_s']), 'steep GBps', round(d['steepest']['k_price_GBps']))" $OUT/bench_$i.json
done
for c in C2 C4 C5; do
  timeout -k 10 600 python3 -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-tableau --no-solve-to-optimum > $OUT/bench_$c.log 2>&1 || { tail -30 $OUT/bench_$c.log; exit 1; }
  grep '^{' $OUT/bench_$c.log > $OUT/bench_$c.json
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); t=d['timed_region']; print(sys.argv[2], round(d['value'],1), 'steps', d['steps'], 'next', [round(v,1) for v in t['next_windows_it_per_s'] or []], 'price frac', round(d['roofline']['frac'],3))" $OUT/bench_$c.json $c
done
