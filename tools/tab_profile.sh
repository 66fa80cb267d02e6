#!/bin/bash
# rocprofv3 kernel-trace stats of the window tableau at C3 (630 pivots = 10
# windows: k_tab_loop passes + k_tab_active + k_tab_fold).  The persistent
# loop kernels are plain launches of a co-resident grid (no cooperative
# launch since r02: a cooperative launch made the process segfault in exit()
# under rocprofv3), so a non-zero rc is a failure like any other.
# usage: tools/tab_profile.sh rNN
set -o pipefail
R=${1:-r02}
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/tabprof_$R"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o tab -- \
    python3 "$ROOT/tools/itbench.py" --tag c3tabprof --k 630 --reps 1 --kw '{"tableau":true}' > "$OUT/tabprof.log" 2>&1 || exit $?
head -8 "$OUT/tab_kernel_stats.csv"
