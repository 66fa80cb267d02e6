#!/bin/bash
# Bench lines of the other BASELINE configs (C2, C4, C5) on one GPU, each the
# last JSON line of `bench.py --config Cx`, written to gpurun_out/cfgs/cN.json.
# usage: tools/cfg_bench.sh [C2 C4 C5]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/cfgs"
mkdir -p "$OUT"
cd "$ROOT"
for c in ${@:-C2 C4 C5}; do
  case $c in
    C2) steps=2000; warm=20 ;;
    C4) steps=126; warm=5 ;;
    C5) steps=126; warm=5 ;;
  esac
  lc=$(echo $c | tr 'C' 'c')
  timeout -k 10 300 python3 -u bench.py --config $c --steps $steps --warmup $warm --no-cpu-baseline --no-tableau \
      > "$OUT/$lc.log" 2>&1 || { tail -20 "$OUT/$lc.log"; exit 1; }
  grep '^{' "$OUT/$lc.log" | tail -1 > "$OUT/$lc.json"
  head -c 400 "$OUT/$lc.json"; echo
done
