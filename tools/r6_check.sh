# Round-6 quick check: ticket-guard / large / deferred-tail GPU tests, then
# fresh-process window timings and two short bench lines.
set -o pipefail
OUT=gpurun_out/${1:-r6b}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_defer.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for p in none none ctx idle; do
  timeout -k 10 120 python3 -u tools/window_fresh.py --pre $p >> $OUT/fresh.jsonl 2>/dev/null || exit 1
done
cut -c1-300 $OUT/fresh.jsonl
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-tableau --no-steepest --no-explicit > $OUT/bench_$i.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); t=d['timed_region']; print(round(d['value']), [round(v) for v in t['next_windows_it_per_s']], round(d['roofline']['frac'],3))" $OUT/bench_$i.json
done
