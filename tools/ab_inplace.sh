#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PP=$PWD/simplex_method_gpu_amd/_build/pp/libsimplex.so
for round in 1 2; do
  for cfg in "4096 16384 200" "16384 65536 40"; do
    set -- $cfg
    timeout -k 10 120 python tools/itbench.py --m $1 --n $2 --k $3 --reps 2 --tag inplace 2>&1 | grep '^{' || exit 1
    SPX_LIB=$PP timeout -k 10 120 python tools/itbench.py --m $1 --n $2 --k $3 --reps 2 --tag pingpong 2>&1 | grep '^{' || exit 1
    timeout -k 10 120 python tools/itbench.py --m $1 --n $2 --k $3 --reps 2 --tag inplace-512x2 --kw '{"update_block":512,"update_rows":2}' 2>&1 | grep '^{' || exit 1
  done
done
