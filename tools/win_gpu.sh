cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests/test_gpu_window.py -x -q -p no:cacheprovider > gpurun_out/win_tests.log 2>&1; rc=$?
echo "window tests rc=$rc"; tail -15 gpurun_out/win_tests.log
[ $rc -eq 0 ] || exit $rc
for w in -1 32 16 64 8; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 400 --warmup 40 --window $w > gpurun_out/bench_w$w.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bench_w$w.log').read().strip().splitlines()[-1]);print('w=$w', round(d['value'],1), 'price_ms', round(d['roofline']['avg_launch_ms'],4), 'upd_ms', round(d['kernels']['k_update']['avg_launch_ms'],4), d['kernels']['iteration'])"
done
