#!/bin/bash
# Sub-phase split of the persistent tableau loop from the diagnostic builds
# (SPX_TAB_CLK=1: column work / barrier 1; SPX_TAB_CLK=2: phase-B prologue).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for M in 0 1 2 3; do
  LIB=$PWD/simplex_method_gpu_amd/_build/libsimplex_clk$M.so
  [ $M -eq 0 ] && LIB=$PWD/simplex_method_gpu_amd/libsimplex.so
  SPX_LIB=$LIB timeout -k 5 60 python tools/loop_probe.py --kw "{\"tableau\":true${TAB_KW}}" --k 189 | sed "s/^/clk$M /" || exit 1
done
