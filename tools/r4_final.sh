# round-4 evidence, part A: every -m gpu test, smoke(), the bench with the
# driver's arguments (3 runs); part B is tools/r4_final_b.sh
set -o pipefail
OUT=gpurun_out/r4final
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
for i in 1 2 3; do
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$i.log 2>&1 || { tail -30 $OUT/bench_$i.log; exit 1; }
grep '^{' $OUT/bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3', d['value'], d['ms_per_step'], d['roofline']['frac'], d['solve_to_optimum']['iterations_per_s'], d['steepest']['solve']['pivots'])"
done
