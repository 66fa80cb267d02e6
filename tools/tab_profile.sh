#!/bin/bash
# rocprofv3 kernel-trace stats of the window tableau at C3 (630 pivots = 10
# windows: k_tab_loop passes + k_tab_fold + k_fold).  Last step of its gpurun
# call: the process segfaults at exit under rocprofv3 after a cooperative
# launch (see tools/gpu_profile.sh), so rc 139 with the stats file written is
# reported as "stats ok, exit crash" and nothing runs after it.
# usage: tools/tab_profile.sh rNN
R=${1:-r01}
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/tabprof_$R"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o tab -- \
    python3 "$ROOT/tools/itbench.py" --tag c3tabprof --k 630 --reps 1 --kw '{"tableau":true}' > "$OUT/tabprof.log" 2>&1
rc=$?
if [ -s "$OUT/tab_kernel_stats.csv" ]; then
    echo "stats ok (rocprofv3 exit rc=$rc)"
    head -8 "$OUT/tab_kernel_stats.csv"
    exit 0
fi
exit $rc
