#!/bin/bash
# update-geometry sweep for the eta-window FTRAN: UPD="1024:1 512:1 256:1" LIBS="default path/to/lib.so"
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; mkdir -p gpurun_out
for lib in ${LIBS:-default}; do for ur in ${UPD:-1024:1 512:1 256:1}; do
  ub=${ur%%:*}; rr=${ur##*:}
  if [ "$lib" = default ]; then unset SPX_LIB; else export SPX_LIB=$lib; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 300 --warmup 80 --window ${W:-64} --update-block $ub --update-rows $rr $BENCH_ARGS > gpurun_out/us.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/us.log').read().strip().splitlines()[-1]);it=d['kernels']['iteration'];print('$lib ub=$ub ur=$rr', round(d['value'],1), 'price_us', round(1e3*d['roofline']['avg_launch_ms'],1), 'upd_us', round(1e3*d['kernels']['k_update']['avg_launch_ms'],1), 'graph_us', round(1e3*it['undisturbed_ms_per_step'],1))"
done; done
