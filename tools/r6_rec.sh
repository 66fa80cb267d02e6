# VERDICT r05 item 3's structural option, built and measured: k_price's last
# workgroup publishes one record (p, its reduced cost, Wt[p][.], A_p on the
# compact list) that k_ftran_bc reads at entry (SPX_PRICE_REC=1, build xrec),
# against the default: the C3 pivot trace (first 300) and pass time.
set -o pipefail
timeout -k 10 300 python3 - <<'PY' || exit 1
import os, subprocess, sys, json
code = r'''
import sys, json, numpy as np
sys.path.insert(0, ".")
import simplex_method_gpu_amd as spx
with spx.Context(m=4096, n=16384, seed=0, device=0, trace=300) as c:
    st, piv = c.iterate(300)
    p, q = c.trace()
    s = c.state()
print(json.dumps({"piv": piv, "p": p.tolist(), "q": q.tolist(), "z": float(np.dot(s["c_B"], s["x_b"]))}))
'''
outs = {}
for lib in ("", os.path.abspath("simplex_method_gpu_amd/_ab/xrec/libsimplex.so")):
    env = dict(os.environ, SPX_LIB=lib) if lib else dict(os.environ)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=200)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if not line:
        print(r.stdout[-500:], r.stderr[-2000:]); sys.exit(1)
    outs[lib or "default"] = json.loads(line[-1])
a, b = outs["default"], outs[[k for k in outs if k != "default"][0]]
print("trace equal", a["p"] == b["p"] and a["q"] == b["q"], "pivots", a["piv"], b["piv"], "z", a["z"], b["z"])
PY
timeout -k 10 600 python3 tools/pass_ab.py default simplex_method_gpu_amd/_ab/xrec/libsimplex.so
