#!/bin/bash
# pricing-geometry sweep under both B^-1 representations (bench, no CPU baseline)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
for w in -1 64; do for pb in 256 512 1024; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 300 --warmup 80 --window $w --price-block $pb $BENCH_ARGS > gpurun_out/ps_$w_$pb.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/ps_$w_$pb.log').read().strip().splitlines()[-1]);it=d['kernels']['iteration'];print('w=$w pb=$pb', round(d['value'],1), 'price_us', round(1e3*d['roofline']['avg_launch_ms'],1), 'upd_us', round(1e3*d['kernels']['k_update']['avg_launch_ms'],1), 'graph_us', round(1e3*it['undisturbed_ms_per_step'],1))"
done; done
