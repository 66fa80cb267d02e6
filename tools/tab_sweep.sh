#!/bin/bash
# Window tableau on the GPU: parity tests, C3 rates (persistent loop, two-kernel
# passes), the loop's phase split, then a rocprofv3 kernel-stats pass (last:
# rocprofv3 has crashed at exit after cooperative launches).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tableau.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tab_tests.log 2>&1; rc=$?
tail -3 gpurun_out/tab_tests.log; [ $rc -eq 0 ] || exit $rc
for kw in '{"tableau":true}' '{"tableau":true,"persist":false}' ${TAB_EXTRA}; do
  timeout -k 10 120 python tools/itbench.py --tag c3tab --k 630 --kw "$kw" || exit $?
  timeout -k 10 120 python tools/loop_probe.py --kw "$kw" --k 189 || exit $?
done
if [ "${TAB_PROF:-0}" = 1 ]; then
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tabprof -o tab -- python3 tools/itbench.py --tag c3tabprof --k 630 --reps 1 --kw '{"tableau":true}' > gpurun_out/tabprof.log 2>&1
  find gpurun_out/tabprof -name "*kernel_stats.csv" -exec head -8 {} \;
fi
exit 0
