#!/bin/bash
# C2 (m=1024 n=4096, latency-bound): explicit / window two-kernel / window persistent.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() { timeout -k 10 120 python tools/itbench.py --m 1024 --n 4096 --k 630 --warm 63 --reps 3 "$@" || exit $?; }
run --tag explicit --kw '{}'
run --tag win64 --kw '{"window":64}'
run --tag win64persist --kw '{"window":64,"persist":true}'
run --tag win32persist --kw '{"window":32,"persist":true}'
timeout -k 10 120 python tools/loop_probe.py --m 1024 --n 4096 --k 126 --kw '{"window":64,"persist":true}' || exit $?
run --m 2048 --n 8192 --tag m2048explicit --kw '{"window":-1}'
run --m 2048 --n 8192 --tag m2048win --kw '{"window":64}'
run --m 2048 --n 8192 --tag m2048persist --kw '{"window":64,"persist":true}'
