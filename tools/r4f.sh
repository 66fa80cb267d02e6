set -o pipefail
OUT=gpurun_out/r4h
mkdir -p $OUT
echo start; date
timeout -k 10 200 python3 -u -c "import torch; print('torch', torch.cuda.is_available())" || exit 1
date
timeout -k 10 90 python3 -u tools/cfold_probe.py > $OUT/cfold_c3.json 2>&1 || { tail -30 $OUT/cfold_c3.json; exit 1; }
date
timeout -k 10 600 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_window.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python3 -u tools/cfold_probe.py --m 16384 --n 65536 > $OUT/cfold_c5.json 2>&1 || { tail -30 $OUT/cfold_c5.json; exit 1; }
timeout -k 10 600 python3 -u tools/pass_ab.py default > $OUT/ab.log 2>&1 || { tail -30 $OUT/ab.log; exit 1; }
tail -1 $OUT/ab.log
