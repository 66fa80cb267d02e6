#!/bin/bash
# Full GPU check for one round step: every -m gpu test, smoke(), the default
# bench line, and the C3 phase probe.  usage: tools/gpu_full.sh TAG
set -o pipefail
T=${1:-full}
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$T"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 400 python3 -u bench.py > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 1; }
grep '^{' "$OUT/bench.log" | tail -1 | head -c 1500; echo
timeout -k 10 120 python3 -u tools/phase_probe.py --variants '[{"window": 64}]' > "$OUT/phase.log" 2>&1 || exit $?
cat "$OUT/phase.log"
