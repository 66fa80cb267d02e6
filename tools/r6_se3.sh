# Where does the steepest-edge solve lose time with the deep prefetch (xs22)?
set -o pipefail
for r in 1 2; do for L in default xs22; do
  if [ $L = default ]; then LIB=""; else LIB=$PWD/simplex_method_gpu_amd/_ab/$L/libsimplex.so; fi
  SPX_LIB=$LIB timeout -k 10 200 python3 tools/se_solve_probe.py || exit 1
done; done
