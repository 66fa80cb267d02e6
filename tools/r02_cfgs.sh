#!/bin/bash
# Bench lines of the other BASELINE configs (C2, C4, C5) on one GPU.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/cfgs"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python3 -u bench.py --config C2 --steps 2000 --warmup 20 --no-cpu-baseline --no-tableau > "$OUT/c2.log" 2>&1 || { tail -20 "$OUT/c2.log"; exit 1; }
grep '^{' "$OUT/c2.log" | tail -1 | head -c 400; echo
timeout -k 10 300 python3 -u bench.py --config C5 --steps 126 --warmup 5 --no-cpu-baseline --no-tableau > "$OUT/c5.log" 2>&1 || { tail -20 "$OUT/c5.log"; exit 1; }
grep '^{' "$OUT/c5.log" | tail -1 | head -c 400; echo
timeout -k 10 300 python3 -u bench.py --config C4 --steps 63 --warmup 5 --no-cpu-baseline --no-tableau > "$OUT/c4.log" 2>&1 || { tail -20 "$OUT/c4.log"; exit 1; }
grep '^{' "$OUT/c4.log" | tail -1 | head -c 400; echo
