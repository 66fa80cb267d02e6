#!/bin/bash
# A/B the cache-policy builds (make variant NT=xyz) on one GPU, interleaved twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2; do
  for v in 000 001 010 011 100 101 110 111; do
    SPX_LIB=$PWD/simplex_method_gpu_amd/_build/v$v/libsimplex.so timeout -k 10 120 python tools/itbench.py --tag v$v --reps 2 2>&1 | grep '^{' || exit 1
  done
done
