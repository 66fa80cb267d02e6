#!/bin/bash
# GPU tests, then the C3 phase probe + iteration rate.  usage: tools/r02_check.sh TAG
set -o pipefail
T=${1:-check}
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$T"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 120 python3 -u tools/phase_probe.py --variants '[{"window": 64}]' > "$OUT/phase.log" 2>&1 || exit $?
cat "$OUT/phase.log"
timeout -k 10 120 python3 -u tools/itbench.py > "$OUT/itbench.log" 2>&1 || exit $?
cat "$OUT/itbench.log"
