#!/bin/bash
# C3 window-tableau rates (persistent loop at several grids vs two-kernel
# passes) + the persistent loop's phase split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tableau.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tab_tests.log 2>&1; rc=$?
tail -3 gpurun_out/tab_tests.log; [ $rc -eq 0 ] || exit $rc
for kw in '{"tableau":true}' '{"tableau":true,"price_grid":96}' '{"tableau":true,"price_grid":128}' '{"tableau":true,"persist":false,"update_block":256,"update_rows":4}' ${TAB_EXTRA}; do
  timeout -k 10 120 python tools/itbench.py --tag c3tab --k 630 --kw "$kw" || exit $?
  timeout -k 10 120 python tools/loop_probe.py --kw "$kw" --k 189 || exit $?
done
