# Steepest-edge k_price A/B, second round: the full two-batch deep prefetch
# made to fit by a 2-element LDS operand batch (SPX_PRICE_DEEP_SE=2
# SPX_SE_LDS_BATCH=2: 248 VGPRs, no spills; build xs22), the batch alone
# (xs02), the default. Pass time, then the bench's steepest block alternating;
# the first 200 steepest-edge pivots' trace compared with the default's.
set -o pipefail
OUT=gpurun_out/${1:-r6se2}
mkdir -p $OUT
timeout -k 10 300 python3 - <<'PY' || exit 1
import os, subprocess, sys, json
code = r'''
import sys, json
sys.path.insert(0, ".")
import simplex_method_gpu_amd as spx
with spx.Context(m=4096, n=16384, seed=0, device=0, trace=200, pricing=spx.PRICING_STEEPEST) as c:
    st, piv = c.iterate(200)
    p, q = c.trace()
    z = c.objective()
print(json.dumps({"p": p.tolist(), "q": q.tolist(), "z": z}))
'''
outs = {}
for name in ("default", "xs22", "xs02"):
    env = dict(os.environ)
    if name != "default":
        env["SPX_LIB"] = os.path.abspath(f"simplex_method_gpu_amd/_ab/{name}/libsimplex.so")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=200)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if not line:
        print(r.stdout[-500:], r.stderr[-2000:]); sys.exit(1)
    outs[name] = json.loads(line[-1])
for name in ("xs22", "xs02"):
    print(name, "trace and z equal to default:", outs[name] == outs["default"])
PY
PASS_AB_PRICING=2 timeout -k 10 500 python3 tools/pass_ab.py default simplex_method_gpu_amd/_ab/xs22/libsimplex.so simplex_method_gpu_amd/_ab/xs02/libsimplex.so || exit 1
for r in 1 2 3; do for L in default xs22 xs02; do
  if [ $L = default ]; then LIB=""; else LIB=$PWD/simplex_method_gpu_amd/_ab/$L/libsimplex.so; fi
  SPX_LIB=$LIB timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-tableau --no-explicit --no-sharded-pricing --no-solve-to-optimum > $OUT/b_${L}_$r.json 2>/dev/null || exit 1
  python3 -c "import json,sys; s=json.load(open(sys.argv[1]))['steepest']; print(sys.argv[2], round(s['k_price_GBps']), round(1e3*s['k_price_ms'],2), 'us', round(s['value']), 'it/s solve', s['solve']['pivots'], round(s['solve']['seconds'],4))" $OUT/b_${L}_$r.json $L
done; done
