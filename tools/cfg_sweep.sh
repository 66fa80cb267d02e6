#!/bin/bash
# representation sweep on other configs: CFGS="C2 C4 C5" WINDOWS="-1 16 64"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
for cfg in ${CFGS:-C2 C4 C5}; do for w in ${WINDOWS:--1 16 64}; do
  steps=300; [ "$cfg" = "C5" ] && steps=60; [ "$cfg" = "C4" ] && steps=120
  timeout -k 10 300 python bench.py --no-cpu-baseline --config $cfg --steps $steps --warmup 70 --window $w > gpurun_out/cs_${cfg}_$w.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/cs_${cfg}_$w.log').read().strip().splitlines()[-1]);it=d['kernels']['iteration'];print('$cfg w=$w', round(d['value'],1), 'price_us', round(1e3*d['roofline']['avg_launch_ms'],1), 'upd_us', round(1e3*d['kernels']['k_update']['avg_launch_ms'],1), 'graph_us', round(1e3*it['undisturbed_ms_per_step'],1), 'event_us', round(1e3*it['event_timed_ms_per_step'],1))"
done; done
