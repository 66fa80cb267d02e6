#!/bin/bash
# rocprofv3 evidence for one round: the bench line alone, the kernel-trace
# stats of the same bench command, two separate PMC passes (FETCH_SIZE,
# WRITE_SIZE) on an eager C3 workload that covers a fold, and the traffic JSON.
# usage: tools/gpu_profile.sh rNN
set -o pipefail
R=${1:-r03}
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/prof_$R"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python3 -u bench.py > "$OUT/bench.log" 2>&1 || exit $?
grep '^{' "$OUT/bench.log" | tail -1 | head -c 600; echo
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --no-sharded-pricing --no-solve-to-optimum --no-steepest > "$OUT/bench_under_rocprof.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o pmc -- \
    python3 "$ROOT/tools/pmc_run.py" --k 110 > "$OUT/pmc_fetch.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o pmc -- \
    python3 "$ROOT/tools/pmc_run.py" --k 110 > "$OUT/pmc_write.log" 2>&1 || exit $?
cd "$ROOT"
python3 tools/pmc_traffic.py "$(find "$OUT/fetch" -name '*counter_collection.csv' | head -1)" \
    "$(find "$OUT/write" -name '*counter_collection.csv' | head -1)" --out "$OUT/traffic_$R.json" || exit $?
find "$OUT" -name "*.csv" | sort
