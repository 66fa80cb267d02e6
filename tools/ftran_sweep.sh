#!/bin/bash
# Eta-window FTRAN variants at C3: A_p in LDS (SPX_WIN_APLDS), loads per round
# trip (SPX_WIN_U1), update geometry.  Build first: make xlib X=apl XFLAGS=...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B=simplex_method_gpu_amd/_build
run() { timeout -k 10 120 python tools/itbench.py "$@" || exit $?; }
for v in default xapl xapl8 xu8 xu32; do
  if [ "$v" = default ]; then lib=""; else lib=$B/$v/libsimplex.so; fi
  for kw in '{}' '{"update_block":1024}' '{"update_block":256}' '{"update_rows":2}'; do
    SPX_LIB=$lib run --tag $v --kw "$kw" --reps 2
  done
done
