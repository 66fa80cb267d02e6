#!/bin/bash
# Diagnostic builds of libsimplex with the tableau loop's stamp at point k
# (SPX_TAB_CLK = k, spx_tableau.hip): _build/libsimplex_clk<k>.so for k in $CLK_MODES.
set -e
cd "$(dirname "$0")/.."
B=simplex_method_gpu_amd/_build
for M in ${CLK_MODES:-1 2 3 4 5 6 7 8 9 10 11}; do
  ( hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -DSPX_TAB_CLK=$M \
      -c simplex_method_gpu_amd/csrc/spx_tableau.hip -o $B/spx_tableau_clk$M.o &&
    hipcc --offload-arch=gfx950 -shared -o $B/libsimplex_clk$M.so $B/spx_kernels.o $B/spx_reinv.o \
      $B/spx_tableau_clk$M.o $B/spx_loop.o $B/spx_api.o -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl ) &
done
wait
