set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "loop or persist or window" > gpurun_out/c5ab_pytest.log 2>&1 || { tail -30 gpurun_out/c5ab_pytest.log; exit 1; }
tail -1 gpurun_out/c5ab_pytest.log
for r in 1 2; do for v in default xprev; do
  if [ $v = default ]; then L=$PWD/simplex_method_gpu_amd/libsimplex.so; else L=$PWD/simplex_method_gpu_amd/_build/$v/libsimplex.so; fi
  SPX_LIB=$L timeout -k 10 200 python tools/itbench.py --tag $v-c5 --m 16384 --n 65536 --k 63 --warm 5 --reps 2 | grep '^{' || exit 1
done; done
