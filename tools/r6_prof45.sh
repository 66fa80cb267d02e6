# rocprofv3 kernel stats of the C4 and C5 bench lines (final build).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/prof45_r06"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for c in C4 C5; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$c" -o bench -- \
      python3 "$ROOT/bench.py" --config $c --no-cpu-baseline --no-sharded-pricing --no-solve-to-optimum --no-steepest --no-tableau --no-explicit > "$OUT/$c.log" 2>&1 || { tail -20 "$OUT/$c.log"; exit 1; }
  grep '^{' "$OUT/$c.log" | tail -1 | head -c 300; echo
  head -4 "$(find "$OUT/$c" -name '*kernel_stats.csv' | head -1)" | cut -c1-160
done
