#!/bin/bash
# Cumulative in-pass profile of the persistent tableau loop: for each
# diagnostic build (tools/build_clk.sh) loop_probe's price_us is the time from
# the pass start to stamp point k (0 = barrier 1 done; see SPX_TAB_CLK in
# spx_tableau.hip), ftran_us from there to barrier 2, tail_us to the next pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for M in 0 ${CLK_MODES:-1 2 3 4 5 6 7 8 9 10 11}; do
  LIB=$PWD/simplex_method_gpu_amd/_build/libsimplex_clk$M.so
  [ $M -eq 0 ] && LIB=$PWD/simplex_method_gpu_amd/libsimplex.so
  SPX_LIB=$LIB timeout -k 5 60 python tools/loop_probe.py --kw "{\"tableau\":true${TAB_KW}}" --k 189 | sed "s/^/clk$M /" || exit 1
done
