#!/bin/bash
# Interleaved A/B of library builds on the C3 window path (tools/itbench.py).
# usage: tools/ab_libs.sh "default xaux2 v100 ..." [rounds]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VS=${1:-default}
for round in $(seq 1 ${2:-2}); do
  for v in $VS; do
    if [ "$v" = default ]; then lib=$PWD/simplex_method_gpu_amd/libsimplex.so; else lib=$PWD/simplex_method_gpu_amd/_build/$v/libsimplex.so; fi
    SPX_LIB=$lib timeout -k 10 120 python tools/itbench.py --tag $v --reps 3 2>&1 | grep '^{' || exit 1
  done
done
