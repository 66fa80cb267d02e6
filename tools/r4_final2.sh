# round-4 final build check after the WM-1-only deep prefetch: every -m gpu
# test, smoke, the C3 bench (driver arguments) and the C5 bench
set -o pipefail
OUT=gpurun_out/r4final2
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c3.log 2>&1 || { tail -30 $OUT/bench_c3.log; exit 1; }
grep '^{' $OUT/bench_c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3', d['value'], d['roofline']['frac'])"
timeout -k 10 500 python3 -u bench.py --gpus 1 --config C5 --steps 126 --warmup 5 --no-cpu-baseline --no-sharded-pricing --no-solve-to-optimum --no-steepest > $OUT/bench_c5.log 2>&1 || { tail -30 $OUT/bench_c5.log; exit 1; }
grep '^{' $OUT/bench_c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5', d['value'], d['roofline']['frac'])"
