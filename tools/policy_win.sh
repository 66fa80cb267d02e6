#!/bin/bash
# Cache-policy A/B of the eta-window path (make variant NT=xyz), interleaved twice.
# usage: tools/policy_win.sh "111 110 100 011 010"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VS=${1:-"111 110 100 011 010"}
for round in 1 2; do
  for v in $VS; do
    if [ "$v" = 111 ]; then lib=$PWD/simplex_method_gpu_amd/libsimplex.so; else lib=$PWD/simplex_method_gpu_amd/_build/v$v/libsimplex.so; fi
    SPX_LIB=$lib timeout -k 10 120 python tools/itbench.py --tag v$v --reps 3 2>&1 | grep '^{' || exit 1
  done
done
