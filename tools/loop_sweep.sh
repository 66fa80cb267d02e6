#!/bin/bash
# Persistent loop variants (make xloop X=...): C3 rate and phase split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B=simplex_method_gpu_amd/_build
timeout -k 10 200 python -m pytest tests/test_gpu_window.py -x -q -p no:cacheprovider > gpurun_out/lsweep_tests.log 2>&1; rc=$?; tail -3 gpurun_out/lsweep_tests.log; [ $rc -eq 0 ] || exit $rc
for v in default ${VARIANTS:-lfu4 lnofpre lfu4nc}; do
  if [ "$v" = default ]; then lib=""; else lib=$B/$v/libsimplex.so; fi
  SPX_LIB=$lib timeout -k 10 120 python tools/itbench.py --tag $v --reps 2 || exit $?
  SPX_LIB=$lib timeout -k 10 120 python tools/loop_probe.py || exit $?
done
timeout -k 10 120 python tools/itbench.py --tag twokernel --kw '{"persist":false}' --reps 2 || exit $?
for v in default ${VARIANTS:-la lb lc ld}; do
  if [ "$v" = default ]; then lib=""; else lib=$B/$v/libsimplex.so; fi
  SPX_LIB=$lib timeout -k 10 200 python tools/itbench.py --m 16384 --n 65536 --k 63 --warm 63 --tag C5$v --reps 1 || exit $?
done
timeout -k 10 200 python tools/itbench.py --m 16384 --n 65536 --k 63 --warm 63 --tag C5twokernel --kw '{"persist":false}' --reps 1 || exit $?
