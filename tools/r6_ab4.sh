# Round-6 A/B session 4: the fused-exchange build against the one before it
# (xold = aa452aa) on the single-GPU C3 / C4 / C5 passes (the fused code is a
# runtime branch compiled into the same instantiations).
set -o pipefail
timeout -k 10 600 python3 tools/pass_ab.py default simplex_method_gpu_amd/_ab/xold/libsimplex.so || exit 1
PASS_AB_M=4096 PASS_AB_N=131072 timeout -k 10 600 python3 tools/pass_ab.py default simplex_method_gpu_amd/_ab/xold/libsimplex.so || exit 1
