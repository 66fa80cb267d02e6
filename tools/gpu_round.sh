# Round GPU check: every -m gpu test, smoke(), then the bench with the driver's
# arguments three times (the timed region's graph builds and the spread of the
# next three windows printed per run).  The per-round rocprofv3 / PMC evidence
# is tools/gpu_profile.sh.
#   tools/gpu_round.sh [bench-only] [OUT_DIR]
set -o pipefail
OUT=${2:-gpurun_out/round}
mkdir -p $OUT
if [ "$1" != "bench-only" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
fi
for i in 1 2 3; do
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$i.log 2>&1 || { tail -30 $OUT/bench_$i.log; exit 1; }
grep '^{' $OUT/bench_$i.log > $OUT/bench_$i.json
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); t=d['timed_region']; print('C3', round(d['value']), round(1e3*d['ms_per_step'], 2), 'us', round(d['roofline']['frac'], 3), 'builds', t['graph_builds'], 'next', [round(v) for v in t['next_windows_it_per_s'] or []], 'to_opt', round(d['solve_to_optimum']['iterations_per_s']))" $OUT/bench_$i.json
done
