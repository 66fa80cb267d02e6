set -o pipefail
mkdir -p gpurun_out/g2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g2/pytest.log 2>&1 || { tail -30 gpurun_out/g2/pytest.log; exit 1; }
tail -2 gpurun_out/g2/pytest.log
for lib in default xbwin1 default xbwin1; do
  if [ $lib = default ]; then L=$PWD/simplex_method_gpu_amd/libsimplex.so; else L=$PWD/simplex_method_gpu_amd/_build/$lib/libsimplex.so; fi
  SPX_LIB=$L timeout -k 10 200 python tools/itbench.py --tag $lib-c4 --m 4096 --n 131072 --k 100 --reps 2 | grep '^{' || exit 1
  SPX_LIB=$L timeout -k 10 200 python tools/itbench.py --tag $lib-c5 --m 16384 --n 65536 --k 60 --warm 5 --reps 2 | grep '^{' || exit 1
  SPX_LIB=$L timeout -k 10 200 python tools/itbench.py --tag $lib-c5-2k --m 16384 --n 65536 --k 60 --warm 5 --reps 2 --kw '{"persist": false}' | grep '^{' || exit 1
done
timeout -k 10 120 python3 -u tools/phase_probe.py --variants '[{"window": 64}]'
