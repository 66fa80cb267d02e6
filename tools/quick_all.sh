#!/bin/bash
# Parity tests, then C2/C3/C4 rates (both B^-1 modes at C3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_window.py tests/test_gpu_parity.py tests/test_gpu_robust.py -x -q -p no:cacheprovider > gpurun_out/quick_tests.log 2>&1; rc=$?; tail -3 gpurun_out/quick_tests.log; [ $rc -eq 0 ] || exit $rc
run() { timeout -k 10 150 python tools/itbench.py --reps 2 "$@" || exit $?; }
run --tag C3 --kw '{}'
run --tag C3explicit --kw '{"window":-1}'
run --m 1024 --n 4096 --k 630 --tag C2 --kw '{}'
run --m 4096 --n 131072 --k 100 --tag C4 --kw '{}'
