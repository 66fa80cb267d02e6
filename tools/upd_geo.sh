#!/bin/bash
# k_update geometry at C3 (window mode, current kernels)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() { timeout -k 10 150 python tools/itbench.py --reps 2 "$@" || exit $?; }
run --tag ub512 --kw '{}'
run --tag ub1024 --kw '{"update_block":1024}'
run --tag ub256 --kw '{"update_block":256}'
run --tag ub512r2 --kw '{"update_rows":2}'
run --tag ub1024r2 --kw '{"update_block":1024,"update_rows":2}'
run --tag pb256 --kw '{"price_block":256}'
run --tag pg512 --kw '{"price_grid":512}'
run --tag pg384 --kw '{"price_grid":384}'
