#!/bin/bash
# GPU tests, then an interleaved A/B of the default build against _build/<variant>
# builds (tools/ab_libs.sh) and the C3 phase probe.  usage: tools/r02_ab.sh TAG "xbase ..."
set -o pipefail
T=${1:-ab}
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$T"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
bash tools/ab_libs.sh "default ${2:-xbase}" 2 > "$OUT/ab.log" 2>&1 || { cat "$OUT/ab.log"; exit 1; }
cat "$OUT/ab.log"
timeout -k 10 120 python3 -u tools/phase_probe.py --variants '[{"window": 64}]' > "$OUT/phase.log" 2>&1 || exit $?
cat "$OUT/phase.log"
