#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2; do
  for v in 111 110 101 100; do
    SPX_LIB=$PWD/simplex_method_gpu_amd/_build/v$v/libsimplex.so timeout -k 10 120 python tools/itbench.py --m 16384 --n 65536 --k 40 --reps 2 --tag v$v --kw '{"update_block":512,"update_rows":2}' 2>&1 | grep '^{' || exit 1
  done
done
for kw in '{"update_block":256,"update_rows":4}' '{"update_block":256,"update_rows":8}' '{"update_block":512,"update_rows":4}' '{"update_block":256,"update_rows":2}' '{"update_block":512,"update_rows":1}'; do
  timeout -k 10 120 python tools/itbench.py --m 16384 --n 65536 --k 40 --reps 2 --kw "$kw" 2>&1 | grep '^{' || exit 1
done
