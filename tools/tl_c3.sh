#!/bin/bash
# rocprofv3 kernel trace of a C3 graph-mode run (tools/itbench.py) and its
# per-kernel / per-seam summary (tools/timeline.py).  usage: tools/tl_c3.sh TAG [itbench args]
set -o pipefail
T=${1:-tl}; shift
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$T"
rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o tl -- \
    python3 "$ROOT/tools/itbench.py" --k 252 --reps 2 "$@" > "$OUT/itbench.log" 2>&1 || exit $?
cd "$ROOT"
python3 tools/timeline.py "$(find "$OUT" -name '*kernel_trace.csv' | head -1)" --skip 300 > "$OUT/timeline.json" || exit $?
head -c 1500 "$OUT/timeline.json"
