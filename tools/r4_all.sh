# round-4 evidence in one call: parts A and B (tools/r4_final.sh, tools/r4_final_b.sh)
set -o pipefail
OUT=gpurun_out/r4final
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
for i in 1 2 3; do
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$i.log 2>&1 || { tail -30 $OUT/bench_$i.log; exit 1; }
grep '^{' $OUT/bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3', d['value'], d['ms_per_step'], d['roofline']['frac'], d['solve_to_optimum']['iterations_per_s'], d['steepest']['solve']['pivots'])"
done
for C in C2 C4 C5; do
X=""; [ $C != C2 ] && X="--no-solve-to-optimum --no-steepest"
timeout -k 10 500 python3 -u bench.py --gpus 1 --config $C --steps 126 --warmup 5 --no-cpu-baseline --no-sharded-pricing $X > $OUT/bench_$C.log 2>&1 || { tail -30 $OUT/bench_$C.log; exit 1; }
grep '^{' $OUT/bench_$C.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$C', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 1000 bash tools/gpu_profile.sh r04 > $OUT/profile.log 2>&1 || { tail -30 $OUT/profile.log; exit 1; }
tail -15 $OUT/profile.log
# k_ftran_bc read attribution: FETCH_SIZE with the chunk-0 / U-row loads trimmed (SPX_FTRAN_TRIM build)
cd /tmp && export TMPDIR=/tmp
SPX_LIB=$GRAFT_REPO_ROOT/simplex_method_gpu_amd/_build/xtrim/libsimplex.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$OUT/fetch_trim -o pmc -- python3 $GRAFT_REPO_ROOT/tools/pmc_run.py --k 110 > $GRAFT_REPO_ROOT/$OUT/pmc_trim.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/pmc_trim.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $OUT/fetch_trim -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY'
import csv, statistics, sys
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(sys.argv[1])) if "k_ftran_bc" in r["Kernel_Name"]][20:]
print("k_ftran_bc FETCH_SIZE (trim build): raw KiB median", statistics.median(v), "x2 bytes", 2048 * statistics.median(v))
PY
