# round GPU check: every -m gpu test, smoke(), the bench with the driver's arguments
# (tools/gpu_round.sh [bench-only])
set -o pipefail
OUT=gpurun_out/round
mkdir -p $OUT
if [ "$1" != "bench-only" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
fi
for i in 1 2 3; do for w in 5 70; do
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup $w > $OUT/bench_w$w.$i.log 2>&1 || { tail -30 $OUT/bench_w$w.$i.log; exit 1; }
grep '^{' $OUT/bench_w$w.$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('warmup', $w, d['value'], d['ms_per_step'], d['roofline']['frac'], d['timed_region'])"
done; done
