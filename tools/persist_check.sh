#!/bin/bash
# Persistent loop kernel: parity tests of the window paths, then C3/C5 rates
# with and without it (SPX_FLAG_NO_PERSIST), both workgroup sizes, phase split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_window.py tests/test_gpu_robust.py -x -q -p no:cacheprovider > gpurun_out/persist_tests.log 2>&1; rc=$?; tail -15 gpurun_out/persist_tests.log; [ $rc -eq 0 ] || exit $rc
run() { timeout -k 10 120 python tools/itbench.py "$@" || exit $?; }
probe() { timeout -k 10 120 python tools/loop_probe.py "$@" || exit $?; }
run --tag persist --kw '{}'
run --tag persist512 --kw '{"loop_block":512}'
run --tag twokernel --kw '{"persist":false}'
probe --kw '{}'
probe --kw '{"loop_block":512}'
run --m 16384 --n 65536 --k 100 --tag C5persist --kw '{}'
probe --m 16384 --n 65536 --k 63 --kw '{}'
