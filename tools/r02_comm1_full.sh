#!/bin/bash
# The whole multi-rank bench (default options, so the explicit block too) and
# the row-sharded variant, each under torch.distributed.run with one rank.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/comm1full
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 \
    bench.py --comm1 --steps 100 > gpurun_out/comm1full/default.log 2>&1 || { tail -30 gpurun_out/comm1full/default.log; exit 1; }
grep '^{' gpurun_out/comm1full/default.log | tail -1 | head -c 700; echo
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29542 \
    bench.py --comm1 --row-shard --steps 100 --no-cpu-baseline > gpurun_out/comm1full/rowshard.log 2>&1 || { tail -30 gpurun_out/comm1full/rowshard.log; exit 1; }
grep '^{' gpurun_out/comm1full/rowshard.log | tail -1 | head -c 700; echo
