#!/bin/bash
# GPU tests, then interleaved itbench A/B of the explicit (-1) and window
# representations, default build vs _build/<variant>.  usage: tools/r02_abexp.sh TAG variant
set -o pipefail
T=${1:-abx}
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$T"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for r in 1 2; do
  for v in default $2; do
    if [ $v = default ]; then L=$ROOT/simplex_method_gpu_amd/libsimplex.so; else L=$ROOT/simplex_method_gpu_amd/_build/$v/libsimplex.so; fi
    SPX_LIB=$L timeout -k 10 120 python3 tools/itbench.py --tag $v-explicit --reps 2 --kw '{"window": -1}' | grep '^{' || exit 1
    SPX_LIB=$L timeout -k 10 120 python3 tools/itbench.py --tag $v-c2 --m 1024 --n 4096 --k 1000 --reps 2 | grep '^{' || exit 1
  done
done
