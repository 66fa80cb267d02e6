#!/bin/bash
# PMC traffic (FETCH_SIZE, WRITE_SIZE: separate passes) of the fold kernels:
# the eta-window k_fold (--k 110 covers one) and the tableau's k_tab_fold
# (two-kernel tableau passes).  usage: tools/pmc_folds.sh rNN
set -o pipefail
R=${1:-r01}
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmcfold_$R"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d "$OUT/win_$c" -o pmc -- \
        python3 "$ROOT/tools/pmc_run.py" --k 110 > "$OUT/win_$c.log" 2>&1 || exit $?
    timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d "$OUT/tab_$c" -o pmc -- \
        python3 "$ROOT/tools/pmc_run.py" --k 110 --tableau > "$OUT/tab_$c.log" 2>&1 || exit $?
done
find "$OUT" -name "*counter_collection.csv" | sort
