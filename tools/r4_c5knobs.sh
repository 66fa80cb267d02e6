set -o pipefail
OUT=gpurun_out/r4c5k
mkdir -p $OUT
B=simplex_method_gpu_amd/_build
PASS_AB_M=16384 PASS_AB_N=65536 timeout -k 10 600 python3 -u tools/pass_ab.py default $B/xnodpp/libsimplex.so $B/xnodeep/libsimplex.so $B/xr3k/libsimplex.so > $OUT/ab_c5.log 2>&1 || { tail -30 $OUT/ab_c5.log; exit 1; }
tail -1 $OUT/ab_c5.log
