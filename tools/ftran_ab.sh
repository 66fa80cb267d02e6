# k_ftran_bc A/B: per build, the PMC FETCH_SIZE / WRITE
# passes of an eager C3 workload (tools/pmc_run.py, 110 pivots) summarised per
# kernel, then the graph time per pass interleaved (tools/pass_ab.py).
#   tools/ftran_ab.sh OUT default xt1 xt2 ...   (xNAME: make xlib X=NAME XFLAGS=...)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$1"; shift
mkdir -p "$OUT"
LIBS=()
for L in "$@"; do
  if [ "$L" = default ]; then LIB=""; LIBS+=(default); else LIB="$ROOT/simplex_method_gpu_amd/_ab/$L/libsimplex.so"; LIBS+=("simplex_method_gpu_amd/_ab/$L/libsimplex.so"); fi
  (cd /tmp && export TMPDIR=/tmp && SPX_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/f_$L" -o pmc -- \
      python3 "$ROOT/tools/pmc_run.py" --k 110 > "$OUT/f_$L.log" 2>&1) || { tail -5 "$OUT/f_$L.log"; exit 1; }
  (cd /tmp && export TMPDIR=/tmp && SPX_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/w_$L" -o pmc -- \
      python3 "$ROOT/tools/pmc_run.py" --k 110 > "$OUT/w_$L.log" 2>&1) || { tail -5 "$OUT/w_$L.log"; exit 1; }
  python3 "$ROOT/tools/pmc_traffic.py" "$(find "$OUT/f_$L" -name '*counter_collection.csv' | head -1)" \
      "$(find "$OUT/w_$L" -name '*counter_collection.csv' | head -1)" --out "$OUT/traffic_$L.json" > /dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['k_ftran_bc']; print(sys.argv[2], 'k_ftran_bc read MB', round(k['read_bytes']/1e6,3), 'raw', round(k['raw_fetch_kib_median']*1.024/1e3,3), 'write MB', round(k['write_bytes']/1e6,3))" "$OUT/traffic_$L.json" "$L"
done
cd "$ROOT" && timeout -k 10 600 python3 tools/pass_ab.py "${LIBS[@]}"
