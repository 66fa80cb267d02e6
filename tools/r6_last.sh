# Last check on HEAD: every -m gpu test, smoke(), the bench with the driver's
# arguments (the driver's own commands, pytest without -s).
set -o pipefail
OUT=gpurun_out/${1:-r6last}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2>/dev/null || exit 1
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); t=d['timed_region']; print('C3', round(d['value']), d['steps'], round(d['roofline']['frac'], 4), d['roofline']['traffic'], 'next', [round(v) for v in t['next_windows_it_per_s']])" $OUT/bench.json
