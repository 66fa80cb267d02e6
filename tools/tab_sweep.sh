#!/bin/bash
# C3 window-tableau rates (persistent loop vs two-kernel passes vs the eta
# window) + kernel stats of the default tableau run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tableau.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tab_tests.log 2>&1; rc=$?
tail -3 gpurun_out/tab_tests.log; [ $rc -eq 0 ] || exit $rc
for kw in '{"tableau":true}' '{"tableau":true,"persist":false,"update_block":256,"update_rows":4}' ${TAB_EXTRA}; do
  timeout -k 10 120 python tools/itbench.py --tag c3tab --k 630 --kw "$kw" || exit $?
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tabprof -o tab -- python3 tools/itbench.py --tag c3tabprof --k 630 --reps 1 --kw '{"tableau":true}' > gpurun_out/tabprof.log 2>&1 || exit $?
find gpurun_out/tabprof -name "*kernel_stats.csv" -exec head -8 {} \;
