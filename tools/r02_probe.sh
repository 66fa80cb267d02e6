#!/bin/bash
# Phase split of the C3 window pass (in-kernel stamps) and a kernel trace of
# graph-mode passes (inter-kernel gaps).  usage: tools/r02_probe.sh TAG
set -o pipefail
T=${1:-probe}
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$T"
mkdir -p "$OUT"
timeout -k 10 120 python3 -u "$ROOT/tools/phase_probe.py" --variants '[{"window": 64}]' > "$OUT/phase.log" 2>&1 || exit $?
cat "$OUT/phase.log"
timeout -k 10 120 python3 -u "$ROOT/tools/itbench.py" > "$OUT/itbench.log" 2>&1 || exit $?
cat "$OUT/itbench.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o it -- \
    python3 "$ROOT/tools/itbench.py" --reps 1 > "$OUT/itbench_rocprof.log" 2>&1 || exit $?
echo trace ok
