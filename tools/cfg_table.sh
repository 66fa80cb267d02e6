#!/bin/bash
# Iteration rate + per-kernel times for C2..C5 in both B^-1 representations
# (DESIGN.md §4b).  One process per line, each under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() { timeout -k 10 240 python tools/itbench.py "$@" || exit $?; }
run --m 1024 --n 4096 --tag C2 --kw '{}'
run --m 4096 --n 16384 --tag C3 --kw '{}'
run --m 4096 --n 16384 --tag C3 --kw '{"window":-1}'
run --m 4096 --n 131072 --tag C4 --kw '{}' --k 100
run --m 4096 --n 131072 --tag C4 --kw '{"window":64}' --k 100
run --m 16384 --n 65536 --tag C5 --kw '{}' --k 100
run --m 16384 --n 65536 --tag C5 --kw '{"window":-1}' --k 100
