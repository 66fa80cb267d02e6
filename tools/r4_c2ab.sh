set -o pipefail
OUT=gpurun_out/r4c2
mkdir -p $OUT
B=simplex_method_gpu_amd/_build
PASS_AB_M=1024 PASS_AB_N=4096 timeout -k 10 300 python3 -u tools/pass_ab.py default $B/xr3k/libsimplex.so > $OUT/ab_c2.log 2>&1 || { tail -30 $OUT/ab_c2.log; exit 1; }
tail -1 $OUT/ab_c2.log
PASS_AB_M=16384 PASS_AB_N=65536 timeout -k 10 500 python3 -u tools/pass_ab.py default $B/xr3k/libsimplex.so > $OUT/ab_c5.log 2>&1 || { tail -30 $OUT/ab_c5.log; exit 1; }
tail -1 $OUT/ab_c5.log
