#!/bin/bash
# rocprofv3 evidence for one round: kernel-trace stats of the bench command and
# two separate PMC passes (FETCH_SIZE, WRITE_SIZE) on the eager workload.
# usage: tools/gpu_profile.sh rNN
# The headline trace runs with --no-tableau: a process that made a cooperative
# launch (the tableau's persistent k_tab_loop) segfaults at exit under
# rocprofv3 after the tool has written its files (tools/tab_exit_probe.py;
# clean without the profiler and with the two-kernel tableau).  The tableau
# trace is tools/tab_profile.sh, its own gpurun call.
set -o pipefail
R=${1:-r01}
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/prof_$R"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
    python3 "$ROOT/bench.py" --steps 200 --warmup 20 --no-cpu-baseline --no-tableau > "$OUT/bench_under_rocprof.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o pmc -- \
    python3 "$ROOT/tools/pmc_run.py" > "$OUT/pmc_fetch.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o pmc -- \
    python3 "$ROOT/tools/pmc_run.py" > "$OUT/pmc_write.log" 2>&1 || exit $?
find "$OUT" -name "*.csv" | sort
