"""Interleaved A/B of library builds (SPX_LIB per subprocess): C3 graph-mode
us per pivot of tools/itbench.py for each build, several rounds.
    python tools/ab_libs.py default simplex_method_gpu_amd/_build/xNAME/libsimplex.so ..."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libs = sys.argv[1:] or ["default"]
res = {l: [] for l in libs}
for r in range(3):
    for l in libs:
        env = dict(os.environ)
        if l != "default":
            env["SPX_LIB"] = os.path.join(ROOT, l)
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "itbench.py"), "--k", "252", "--reps", "3"],
                             capture_output=True, text=True, env=env, timeout=300)
        line = [x for x in out.stdout.splitlines() if x.startswith("{")]
        if not line:
            print(out.stdout[-500:], out.stderr[-1500:], flush=True)
            sys.exit(1)
        d = json.loads(line[-1])
        res[l].append(min(d["ms_per_iter"]) * 1e3)
        print(json.dumps({"lib": l, "us_per_pivot": round(res[l][-1], 2), "update_us": d["update_us"],
                          "price_us": d["price_us"]}), flush=True)
print(json.dumps({l: round(min(v), 2) for l, v in res.items()}))
