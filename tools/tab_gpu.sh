#!/bin/bash
# Window tableau on the GPU: its parity tests, then C3 rates (tableau vs eta
# window) and a rocprofv3 kernel-stats pass of the tableau run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tableau.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tab_tests.log 2>&1; rc=$?
tail -15 gpurun_out/tab_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/itbench.py --tag c3tab --k 630 --kw '{"tableau":true}' || exit $?
timeout -k 10 120 python tools/itbench.py --tag c3win --k 630 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tabprof -o tab -- python3 tools/itbench.py --tag c3tabprof --k 630 --reps 1 --kw '{"tableau":true}' > gpurun_out/tabprof.log 2>&1 || exit $?
find gpurun_out/tabprof -name "*kernel_stats.csv" -exec head -12 {} \;
