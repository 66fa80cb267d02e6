set -o pipefail
OUT=gpurun_out/r4prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-sharded-pricing --no-solve-to-optimum --no-steepest > $GRAFT_REPO_ROOT/$OUT/bench_under_rocprof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/bench_under_rocprof.log; exit 1; }
cd $GRAFT_REPO_ROOT
cut -d, -f1-4 $OUT/trace/bench_kernel_stats.csv | head -12
