#!/bin/bash
# Quick A/B: window + parity tests, then C3 rate and phase split of the two-kernel pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_window.py tests/test_gpu_parity.py -x -q -p no:cacheprovider > gpurun_out/quick_tests.log 2>&1; rc=$?; tail -3 gpurun_out/quick_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/itbench.py --tag c3 --reps 3 || exit $?
timeout -k 10 120 python tools/itbench.py --tag c3explicit --kw '{"window":-1}' --reps 2 || exit $?
timeout -k 10 120 python tools/phase_probe.py || exit $?
