#!/bin/bash
# eta-window check: window tests, bench sweep over representations, rocprof trace of one window bench
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests/test_gpu_window.py -x -q -p no:cacheprovider > gpurun_out/win_tests.log 2>&1; rc=$?
echo "window tests rc=$rc"; tail -3 gpurun_out/win_tests.log
[ $rc -eq 0 ] || exit $rc
for w in ${WINDOWS:--1 8 16 32 64}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 400 --warmup 40 --window $w $BENCH_ARGS > gpurun_out/bench_w$w.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bench_w$w.log').read().strip().splitlines()[-1]);it=d['kernels']['iteration'];print('w=$w', round(d['value'],1), 'price_us', round(1e3*d['roofline']['avg_launch_ms'],1), 'upd_us', round(1e3*d['kernels']['k_update']['avg_launch_ms'],1), 'event_us', round(1e3*it['event_timed_ms_per_step'],1), 'graph_us', round(1e3*it['undisturbed_ms_per_step'],1))"
done
PW=${PROF_WINDOW:-32}
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_w$PW" -o bench -- \
    python3 "$ROOT/bench.py" --steps 300 --warmup 40 --no-cpu-baseline --window $PW $BENCH_ARGS > "$ROOT/gpurun_out/prof_w$PW.log" 2>&1 || exit $?
f=$(find "$ROOT/gpurun_out/prof_w$PW" -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f" | head -12
